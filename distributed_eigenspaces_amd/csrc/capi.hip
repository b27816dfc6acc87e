// extern "C" boundary of libdeig.so (declared in include/deig.h) and the host
// drivers of the two eigensolvers.  No device allocation happens here: all
// device memory is caller-provided (PyTorch tensors on the Python side).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#include <algorithm>

#include "deig_internal.hpp"

namespace deig {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int num_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return 256;  // MI355X; only reached by workspace queries without a device
  }
  if (!cache[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0) {
      (void)hipGetLastError();
      v = 256;
    }
    cache[dev] = v;
  }
  return cache[dev];
}

namespace {

constexpr int kMaxP = 128;
// Stagnation handling of the solver (see solve()): a stalled residual counts as
// converged when <= max(kStallAcceptTol * tol, kStallAcceptAbs) - the fp32 floor
// of ||S v - lambda v|| / |lambda_max| is a few 1e-7 up to d = 16384 - and the
// solver gives up after kStallGiveUp Rayleigh-Ritz steps without a 10% gain.
constexpr float kStallAcceptTol = 4.0f;
constexpr float kStallAcceptAbs = 2e-6f;
constexpr int kStallGiveUp = 12;
// Deflation stage of the explicit-matrix solver (see solve()): eigenpairs with
// theta_j >= kDeflateRatio * theta_{k-1} (at most kMaxDeflate of them) are
// deflated out of the sweep image and the rest iterated again.
constexpr float kDeflateRatio = 64.f;
constexpr int kMaxDeflate = 8;

struct Operator {
  bool implicit;
  const float* S;
  int64_t lds;
  const float* Wt;
  int64_t mk, ldw;
  float scale;
};

struct SolverWs {
  RRBuffers rr;
  float* Zt;
  float* T;  // d x p: X_{j-1} of the Chebyshev recurrence
  float* slab;
  size_t slab_bytes;
  void* sweep_ws;  // bf16x6 sweep (explicit S only)
  size_t sweep_bytes;
};

// Sweep algorithm of the explicit-matrix solver: DEIG_SWEEP_ALGO=fp32 selects the
// f32 MFMA skinny kernel, anything else the bf16x6 sweep (sweep.hip).
int sweep_algo_default() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DEIG_SWEEP_ALGO");
    v = (e && strcmp(e, "fp32") == 0) ? DEIG_SWEEP_FP32 : DEIG_SWEEP_BF16X6;
  }
  return v;
}

SolverWs carve_solver(void* ws, size_t cap, int64_t d, int k, int p, int64_t mk, size_t* total) {
  Carve c(ws, cap);
  SolverWs w;
  w.rr.Z = c.take<float>((size_t)d * 2 * p);
  w.rr.C = c.take<float>((size_t)4 * p * p);
  w.rr.Linv = c.take<float>((size_t)p * p);
  w.rr.Wtmp = c.take<float>((size_t)p * p);
  w.rr.W = c.take<float>((size_t)p * p);
  w.rr.lam = c.take<float>((size_t)p);
  w.rr.cs = c.take<float>((size_t)p);
  w.rr.qs = c.take<float>((size_t)p);
  w.rr.resid_part = c.take<float>((size_t)rr_update_blocks(d) * k);
  w.rr.resid = c.take<float>((size_t)k + 1);
  w.rr.info = c.take<int>(16);
  w.Zt = mk > 0 ? c.take<float>((size_t)mk * p) : nullptr;
  w.T = c.take<float>((size_t)d * p);
  size_t sb = skinny_workspace_bytes(2 * p, 2 * p, d);  // Gram
  if (mk > 0) {
    const size_t a = skinny_workspace_bytes(mk, p, d);  // Wt Q
    const size_t b = skinny_workspace_bytes(d, p, mk);  // Wt^T Zt
    if (a > sb) sb = a;
    if (b > sb) sb = b;
  } else {
    const size_t a = skinny_workspace_bytes(d, p, d);  // S Q
    if (a > sb) sb = a;
  }
  w.slab = c.take<float>(sb / sizeof(float) + 4);
  w.slab_bytes = sb;
  w.sweep_ws = nullptr;
  w.sweep_bytes = 0;
  if (mk == 0 && sweep_algo_default() == DEIG_SWEEP_BF16X6) {
    w.sweep_bytes = sweep_workspace_bytes(d, p);
    w.sweep_ws = c.take<char>(w.sweep_bytes);
  }
  *total = c.off;
  return w;
}

// Y = A Q without a sweep image: the fp32 skinny product (explicit S) or the
// implicit projector average Wt^T (Wt Q) (the server).
int apply_op_plain(const Operator& op, const SolverWs& w, int64_t d, int p, hipStream_t st) {
  float* Q = w.rr.Z;
  float* Y = w.rr.Z + p;
  const int64_t ld = 2 * p;
  if (!op.implicit)
    return skinny_launch(true, op.S, op.lds, Q, ld, Y, ld, d, p, d, 1.f, 0.f, w.slab,
                         w.slab_bytes, st);
  int rc = skinny_launch(false, op.Wt, op.ldw, Q, ld, w.Zt, p, op.mk, p, d, 1.f, 0.f, w.slab,
                         w.slab_bytes, st);
  if (rc) return rc;
  return skinny_launch(true, op.Wt, op.ldw, w.Zt, p, Y, ld, d, p, op.mk, op.scale, 0.f, w.slab,
                       w.slab_bytes, st);
}

// Y = A Q.  step (optional): the basis step that follows (power / Chebyshev).  On
// the sweep path it is fused into the sweep's split-K reduction together with the
// next sweep's Q image, and q_ready says that this sweep's image was written by
// the previous one (sweep.hip sweep_finish_kernel); elsewhere it runs as its own
// kernel after the product.
int apply_op(const Operator& op, const SolverWs& w, int64_t d, int p, hipStream_t st, int smode,
             const SweepStep* step = nullptr, bool q_ready = false) {
  float* Q = w.rr.Z;
  float* Y = w.rr.Z + p;
  const int64_t ld = 2 * p;
  if (!op.implicit && w.sweep_ws)
    return sweep_apply(op.S, d, op.lds, Q, p, ld, Y, ld, 1.f, w.sweep_ws, w.sweep_bytes, st,
                       smode, step, q_ready);
  int rc = apply_op_plain(op, w, d, p, st);
  if (rc || !step) return rc;
  if (step->kind == 1) return rr_power_launch(w.rr, d, p, step->tau, st);
  return cheb_step_launch(w.rr, w.T, d, p, step->thr, step->a, step->cc, step->gamma, st);
}

// Whether apply_op fuses steps and Q images (the q_ready protocol applies).
bool fused_steps(const Operator& op, const SolverWs& w) { return !op.implicit && w.sweep_ws; }


// Chebyshev filter plan for the sweeps between two Rayleigh-Ritz steps (host side,
// from the last RR's Ritz values theta_0 >= ... >= theta_{p-1} and residual).
// The operator is assumed PSD (covariances, projector averages): the damped
// interval is [0, c] with c = theta_{p-1} (the block's smallest Ritz value) when
// the basis has guard columns, else min(theta_{p-1}, theta_{k-1} / 2).  Scaled
// recurrence at gamma = theta_0 (Zhou & Saad): X_1 = (s1/e)(A - cc) X_0,
// X_{j+1} = (2 s_{j+1}/e)(A - cc) X_j - s_j s_{j+1} X_{j-1}, s_{j+1} = 1/(2/s1 - s_j).
// Degree m: at most kChebMaxDeg, at most what the residual still needs at column
// k's damping rate, and small enough that a column's contamination by theta_0's
// direction grows at most gmax = clamp(1/resid, 10, kChebGmax) times (the fp32
// Gram of the filtered block must still resolve every column); columns whose
// growth would exceed gmax stay out of the filter (threshold thr on theta_j).
// Only used once resid <= kChebAbove: before that the Ritz values are too rough
// to place the interval, and plain power steps run.
constexpr float kChebAbove = 1e-2f;
float cheb_above() {  // DEIG_CHEB_ABOVE overrides (A/B)
  static const float v = getenv("DEIG_CHEB_ABOVE") ? (float)atof(getenv("DEIG_CHEB_ABOVE")) : kChebAbove;
  return v;
}
constexpr double kChebGmax = 1e4;
constexpr int kChebMaxDeg = 16;

struct ChebPlan {
  int m = 0;
  double cc = 0, e = 1, s1 = 0;
  float thr = 0;
};

bool cheb_plan(const float* lam, int k, int p, float resid, float tol, ChebPlan* pl) {
  if (!(resid <= cheb_above()) || !(resid > 0)) return false;
  const double gmax = fmin(kChebGmax, fmax(10.0, 1.0 / (double)resid));
  const double a = 0.0;
  double c = lam[p - 1];
  if (p - k < 4) c = fmin(c, 0.5 * (double)lam[k - 1]);
  const double lk = lam[k - 1], l0 = lam[0];
  if (!(lk > c && c > a && l0 > c)) return false;
  const double cc = 0.5 * (c + a), e = 0.5 * (c - a);
  const double tk = (lk - cc) / e, t0 = (l0 - cc) / e;
  const double ak = acosh(tk), a0 = acosh(t0);
  const double rho = 1.0 / (tk + sqrt(tk * tk - 1.0));  // column k's damping per degree
  int m = kChebMaxDeg;
  if (a0 - ak > 1e-9) m = std::min(m, std::max(1, (int)(log(gmax) / (a0 - ak))));
  const double need = log(fmax(0.3 * (double)tol / (double)resid, 1e-30)) / log(rho);
  m = std::max(1, std::min(m, (int)ceil(need)));
  pl->m = m;
  pl->cc = cc;
  pl->e = e;
  pl->s1 = 1.0 / t0;
  pl->thr = (float)(cc + cosh(fmax(a0 - log(gmax) / m, 0.0)) * e);
  return true;
}

int solve(const Operator& op, int64_t d, int k, int p, int max_sweeps, float tol, const float* Q0,
          int k0, int64_t ldq0, float* V, int64_t ldv, float* evals, int* sweeps_out,
          float* resid_out, void* ws, size_t ws_bytes, hipStream_t st) {
  DEIG_REQUIRE(d >= 16 && d % 4 == 0, "solver: d=%lld must be >= 16 and a multiple of 4",
               (long long)d);
  DEIG_REQUIRE(k >= 1 && k <= d, "solver: need 1 <= k <= d (k=%d, d=%lld)", k, (long long)d);
  if (p <= 0) p = deig_default_subspace(d, k);
  DEIG_REQUIRE(p % 16 == 0 && p >= k && p <= kMaxP && p <= d,
               "solver: subspace p=%d must be a multiple of 16 with k <= p <= min(128, d)", p);
  DEIG_REQUIRE(max_sweeps >= 1, "solver: max_sweeps must be >= 1");
  DEIG_REQUIRE(V && evals && ldv >= d, "solver: bad V / evals / ldv");
  DEIG_REQUIRE(k0 >= 0 && k0 <= p && (k0 == 0 || (Q0 && ldq0 >= d)), "solver: bad warm start");
  size_t total = 0;
  SolverWs w = carve_solver(ws, ws_bytes, d, k, p, op.implicit ? op.mk : 0, &total);
  if (!ws || total > ws_bytes)
    return fail(DEIG_EWORKSPACE, "solver: workspace %zu bytes < required %zu", ws_bytes, total);

  static const bool debug = getenv("DEIG_DEBUG") && getenv("DEIG_DEBUG")[0] == '1';
  // Cycles: [filter / power sweeps] + one sweep with a Rayleigh-Ritz step (Gram +
  // small solve + update + residual check).  Between two RRs either a Chebyshev
  // filter of planned degree runs (cheb_plan; DEIG_CHEB=0 disables it) or, while
  // the residual is above kChebAbove, rr_every - 1 plain power steps Q <- A Q on
  // the Ritz vectors of the last RR (same span as subspace iteration; the
  // generalised RR copes with the non-orthonormal basis).  The single-workgroup
  // small solve is the latency-bound part of a cycle, so spacing RRs divides its
  // cost.  Power steps: every 4th sweep is an RR when the basis has >= 16 guard
  // columns beyond k (measured: d=8192 k=64 p=80 6.2 vs 9.0 ms, d=3072 k=16 p=32
  // 1.4 vs 1.9 ms); every 2nd without them (d=16384 k=128 p=128: 23 sweeps /
  // 47 ms vs 41 / 54 ms).
  static const int rr_every_env = getenv("DEIG_RR_EVERY") ? atoi(getenv("DEIG_RR_EVERY")) : 0;
  static const bool cheb_on = !(getenv("DEIG_CHEB") && getenv("DEIG_CHEB")[0] == '0');
  const int rr_every = rr_every_env > 0 ? rr_every_env : (p - k >= 16 ? 4 : 2);
  const float tau = rr_every > 1 ? powf(0.1f, 1.0f / (float)(rr_every - 1)) : 0.f;
  int rc = rr_init_launch(w.rr.Z, d, p, Q0, k0, ldq0, 0x5eed5eedull, st);
  if (rc) return rc;
  if (!op.implicit && w.sweep_ws &&
      (rc = sweep_prepare(op.S, d, op.lds, p, w.sweep_ws, w.sweep_bytes, st)))
    return rc;
  float lam_h[kMaxP];
  float res_h[kMaxP + 1];  // per-column residuals of the last RR (descending Ritz order)
  int jconv_h = 1;         // the last RR's Jacobi converged (rr.hip info[3])
  int it = 0;  // sweeps done (both stages)
  float last = 3.4e38f;
  bool converged = false;
  // Stage 1 may end as soon as the dominant pairs that stage 2 deflates are
  // converged (their own residuals <= tol), instead of waiting for every column:
  // with theta_0 ~ 10^4 theta_k (uncentered data) the Chebyshev filter of stage 1
  // is held to degree 1 by the dominant direction's growth bound, so its later
  // cycles are one sweep per Rayleigh-Ritz step.  DEIG_DEFLATE_EARLY=0: off.
  static const bool deflate_on = !(getenv("DEIG_DEFLATE") && getenv("DEIG_DEFLATE")[0] == '0');
  static const bool deflate_early =
      !(getenv("DEIG_DEFLATE_EARLY") && getenv("DEIG_DEFLATE_EARLY")[0] == '0');
  const bool can_deflate = deflate_on && !op.implicit && w.sweep_ws && sweep_version() != 1 && k >= 2;
  auto dominant = [&](int kk) {  // pairs stage 2 would deflate (0: none)
    if (!(lam_h[kk - 1] > 0.f && lam_h[0] >= kDeflateRatio * lam_h[kk - 1])) return 0;
    int r = 0;
    while (r < kk - 1 && r < kMaxDeflate && lam_h[r] >= kDeflateRatio * lam_h[kk - 1]) ++r;
    return r;
  };
  bool early = false;
  // Sweeps round Q to two bf16 pieces (five products instead of six, sweep.hip
  // split_q_kernel) while the residual is above round_until: the rounding puts
  // ~4e-6 relative noise into the basis each sweep, harmless while the Ritz
  // vectors are far from converged, but a floor under the residual, so the
  // closing sweeps use the exact (3-piece) Q.
  // Worker solves (explicit S): 2 sweeps while the residual is above 1e-4 (r02s A/B,
  // profiles/r02s_jacobi_cap_ab.log: c1 +8 %, c1g +14 % over 3 above 1e-2, c3 the
  // same time in 16 sweeps instead of 12; 1 sweep fails the bars).  The server's
  // implicit projector average (eigenvalues clustered near 1) keeps 3 above 1e-2:
  // there the tighter cap cost config 4's aggregation 2.05 -> 2.65 ms.
  static const int jcap_env =
      getenv("DEIG_JACOBI_EARLY") ? atoi(getenv("DEIG_JACOBI_EARLY")) : -1;
  static const float jcap_above_env =
      getenv("DEIG_JACOBI_EARLY_ABOVE") ? (float)atof(getenv("DEIG_JACOBI_EARLY_ABOVE")) : -1.f;
  const int jcap_sweeps = jcap_env >= 0 ? jcap_env : (op.implicit ? 3 : 2);
  const float jcap_above = jcap_above_env >= 0.f ? jcap_above_env : (op.implicit ? 1e-2f : 1e-4f);
  // Early sweeps (residual above fast_until) take S as its two leading bf16 pieces
  // too: three products, no split in the sweep, ~2^-16 relative - 100x below the
  // residual there (sweep.hip sweep_products SP = 2).  DEIG_SWEEP_FAST_UNTIL=0: off.
  static const float fast_until =
      getenv("DEIG_SWEEP_FAST_UNTIL") ? (float)atof(getenv("DEIG_SWEEP_FAST_UNTIL")) : 1e-3f;
  static const float round_until =
      getenv("DEIG_SWEEP_ROUND_UNTIL") ? (float)atof(getenv("DEIG_SWEEP_ROUND_UNTIL")) : 1e-4f;

  // One stage of the iteration for the top kc pairs (V / evals columns 0..kc-1).
  // Returns a status; sets converged / last; advances it.
  auto iterate = [&](int kc) -> int {
    float best = 3.4e38f;
    int since_best = 0;
    int nrr = 0;
    last = 3.4e38f;
    converged = false;
    while (it < max_sweeps) {
      const int smode = (fast_until > 0.f && last > fmaxf(fast_until, tol)) ? kSweepFast
                        : last > fmaxf(round_until, tol)                 ? kSweepRoundQ
                                                                         : kSweepExact;
      ChebPlan plan;
      const bool cheb = cheb_on && nrr > 0 && cheb_plan(lam_h, kc, p, last, tol, &plan);
      int ncheb = 0, nstep = 0, rc2;
      // every sweep of a cycle runs in smode, so a fused step can write the next
      // sweep's Q image (q_ready from the second sweep of the cycle on)
      const bool fuse = fused_steps(op, w);
      SweepStep step{};
      step.Q = w.rr.Z;
      step.ldq = 2 * p;
      step.T = w.T;
      step.cs = w.rr.cs;
      step.lam = w.rr.lam;
      step.next_mode = smode;
      if (cheb) {
        // degree j: apply A to X_j, then X_{j+1} from X_j, A X_j and X_{j-1}
        const int m = std::min(plan.m, max_sweeps - it - 1);
        double s_prev = plan.s1;
        for (int j = 0; j < m; ++j, ++it, ++nstep) {
          double alpha, gamma;
          if (j == 0) {
            alpha = plan.s1 / plan.e;
            gamma = 0.0;
          } else {
            const double s_next = 1.0 / (2.0 / plan.s1 - s_prev);
            alpha = 2.0 * s_next / plan.e;
            gamma = s_prev * s_next;
            s_prev = s_next;
          }
          step.kind = 2;
          step.thr = plan.thr;
          step.a = (float)alpha;
          step.cc = (float)plan.cc;
          step.gamma = (float)gamma;
          if ((rc2 = apply_op(op, w, d, p, st, smode, &step, fuse && nstep > 0))) return rc2;
        }
        ncheb = m;
      } else if (nrr > 0) {
        const int npow = std::min(rr_every - 1, max_sweeps - it - 1);
        // power steps on the live Ritz columns of the last RR (Q_j <- Y_j / ||Y w_j||)
        step.kind = 1;
        step.tau = tau;
        for (int j = 0; j < npow; ++j, ++it, ++nstep)
          if ((rc2 = apply_op(op, w, d, p, st, smode, &step, fuse && nstep > 0))) return rc2;
      }
      if ((rc2 = apply_op(op, w, d, p, st, smode, nullptr, fuse && nstep > 0))) return rc2;
      ++it;
      if ((rc2 = skinny_launch(true, w.rr.Z, 2 * p, w.rr.Z, 2 * p, w.rr.C, 2 * p, 2 * p, 2 * p,
                               d, 1.f, 0.f, w.slab, w.slab_bytes, st)))
        return rc2;
      // Early Rayleigh-Ritz steps (residual above jcap_above) run a capped number
      // of Jacobi sweeps: the next basis Y W spans span(Y) for any invertible W, so
      // subspace progress does not need converged Ritz vectors there; the residual
      // of approximate pairs only over-states the error (no false convergence).
      const int jcap = (jcap_sweeps > 0 && last > jcap_above) ? jcap_sweeps : 30;
      if ((rc2 = rr_small_launch(w.rr, p, st, jcap))) return rc2;
      if ((rc2 = rr_update_launch(w.rr, d, p, kc, V, ldv, evals, st))) return rc2;
      DEIG_HIP_CHECK(
          hipMemcpyAsync(res_h, w.rr.resid, sizeof(float) * (kc + 1), hipMemcpyDeviceToHost, st));
      DEIG_HIP_CHECK(hipMemcpyAsync(lam_h, w.rr.lam, sizeof(float) * p, hipMemcpyDeviceToHost, st));
      jconv_h = 1;
      if (jcap < 30)
        DEIG_HIP_CHECK(
            hipMemcpyAsync(&jconv_h, w.rr.info + 3, sizeof(int), hipMemcpyDeviceToHost, st));
      DEIG_HIP_CHECK(hipStreamSynchronize(st));
      last = res_h[kc];
      // Ritz pairs of a capped Jacobi that stopped short are approximate: their
      // residual bounds the error, but the eigenvalues / vectors returned are those
      // of an unconverged small solve, so no exit is taken on them - the next RR
      // (the residual is then below jcap_above) runs the Jacobi to convergence.
      // Needed where the residual is relative to a dominant theta_0 (worker S:
      // r02s, a 2-sweep cap at every residual missed a CIFAR-gray eigenvalue by
      // 1.0046e-5); the server's projector average (eigenvalues in [0, 1], top k
      // near 1) exits as before - guarding it cost c1's server 5 -> 7 sweeps.
      const bool exact_rr = jconv_h != 0 || op.implicit;
      ++nrr;
      if (debug) {
        int inf[9] = {0};
        DEIG_HIP_CHECK(hipMemcpy(inf, w.rr.info, sizeof(inf), hipMemcpyDeviceToHost));
        fprintf(stderr, "[deig] d=%lld k=%d p=%d sweep %d resid %.3e cheb_deg %d chol_floor %d "
                "jacobi_sweeps %d rotations %d small-solve us: chol %.1f linv %.1f congr %.1f "
                "jacobi %.1f tail %.1f\n",
                (long long)d, kc, p, it, last, ncheb, inf[0], inf[1], inf[2], inf[4] * 0.01,
                (inf[5] - inf[4]) * 0.01, (inf[6] - inf[5]) * 0.01, (inf[7] - inf[6]) * 0.01,
                (inf[8] - inf[7]) * 0.01);
      }
      if (!(last == last) || last > 3.0e38f)  // NaN / Inf
        return fail(DEIG_EINVAL, "solver: non-finite residual (input contains NaN/Inf?)");
      if (!exact_rr) continue;
      if (last <= tol) {
        converged = true;
        return DEIG_OK;
      }
      if (kc == k && can_deflate && deflate_early && last == last) {
        const int r = dominant(k);
        bool ok = r >= 1;
        for (int j = 0; j < r && ok; ++j) ok = res_h[j] <= tol;
        if (ok) {
          early = true;
          return DEIG_OK;
        }
      }
      // Stagnation: no 10% improvement over the best residual for 4 Rayleigh-Ritz
      // steps in a row.  It counts as convergence only at the fp32 floor (residual
      // within kStallAccept* of tol); a stall above it is slow convergence (a small
      // eigengap at k), so the iteration goes on and, if it stays stuck for
      // kStallGiveUp RR steps, stops early with DEIG_NOT_CONVERGED.
      if (last < 0.9f * best) {
        best = last;
        since_best = 0;
      } else if (++since_best >= 4 && it >= 8) {
        if (last <= fmaxf(kStallAcceptTol * tol, kStallAcceptAbs)) {
          converged = true;
          return DEIG_OK;
        }
        if (since_best >= kStallGiveUp) return DEIG_OK;
      }
    }
    return DEIG_OK;
  };

  rc = iterate(k);
  if (rc) {
    if (sweeps_out) *sweeps_out = it;
    if (resid_out) *resid_out = last;
    return rc;
  }
  // Stage 2 - deflation of dominant eigenpairs.  With theta_0 >> theta_{k-1} (an
  // uncentered covariance: the mean direction dwarfs the rest, as for the
  // reference's CIFAR bytes) every fp32 product S q loses ~log2(theta_0 / theta_k)
  // bits of the small eigenvalues' directions to cancellation, which caps their
  // accuracy far above the residual test's reach (relative to theta_0).  The r
  // leading pairs with theta_j >= kDeflateRatio theta_{k-1} are then accurate
  // (huge gap), so the sweep image is rebuilt as S - V_D Lam_D V_D^T and the
  // remaining k - r pairs are iterated again from their current values (warm
  // start), with the residual now relative to theta_r.  V_D stays in the last r
  // columns of V (ascending order), which the second stage does not touch.
  if (can_deflate && (converged || early) && dominant(k) >= 1) {
    const int r = dominant(k);
    const int kc = k - r;
    const float* Vd = V + (int64_t)kc * ldv;
    if ((rc = sweep_prepare(op.S, d, op.lds, p, w.sweep_ws, w.sweep_bytes, st, Vd, ldv,
                            evals + kc, r)))
      return rc;
    if ((rc = rr_init_launch(w.rr.Z, d, p, V, kc, ldv, 0x5eed5eefull, st))) return rc;
    rc = iterate(kc);
    if (!rc) rc = deflate_orth_launch(V, ldv, d, kc, r, st);
    if (debug)
      fprintf(stderr, "[deig] deflated %d dominant pair(s)%s: stage 2 resid %.3e after %d sweeps\n",
              r, early ? " (early)" : "", last, it);
    if (rc) {
      if (sweeps_out) *sweeps_out = it;
      if (resid_out) *resid_out = last;
      return rc;
    }
  }
  if (sweeps_out) *sweeps_out = it;
  if (resid_out) *resid_out = last;
  if (!converged)
    return fail(DEIG_NOT_CONVERGED, "solver: residual %g > tol %g after %d sweeps%s", last, tol,
                it, it < max_sweeps ? " (stalled: eigengap at k too small for the subspace)" : "");
  return DEIG_OK;
}

}  // namespace
}  // namespace deig

using namespace deig;

extern "C" {

int deig_version(void) { return 0x000100; }

const char* deig_last_error(void) { return g_err; }

static int syrk_resolve(int64_t n, int algo) {
  if (algo != DEIG_SYRK_AUTO) return algo;
  return n >= DEIG_SYRK_SPLIT_MIN_ROWS ? DEIG_SYRK_SPLIT3 : DEIG_SYRK_FP32;
}

size_t deig_syrk_workspace_ex(int64_t n, int64_t d, int algo) {
  algo = syrk_resolve(n, algo);
  if (algo == DEIG_SYRK_FP32) return syrk_workspace_bytes(n, d);
  if (algo == DEIG_SYRK_SPLIT3) return syrk_split_workspace_bytes(n, d);
  return 0;
}

int deig_syrk_f32_ex(const float* X, int64_t n, int64_t d, int64_t ldx, float alpha, float* S,
                     int64_t lds, int algo, void* ws, size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  algo = syrk_resolve(n, algo);
  if (algo == DEIG_SYRK_FP32)
    return syrk_launch(X, n, d, ldx, alpha, S, lds, ws, ws_bytes, (hipStream_t)stream);
  if (algo == DEIG_SYRK_SPLIT3)
    return syrk_split_launch(X, n, d, ldx, alpha, S, lds, ws, ws_bytes, (hipStream_t)stream);
  return fail(DEIG_EINVAL, "syrk: unknown algorithm %d", algo);
}

size_t deig_syrk_workspace(int64_t n, int64_t d) {
  return deig_syrk_workspace_ex(n, d, DEIG_SYRK_DEFAULT);
}

int deig_syrk_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float alpha, float* S,
                  int64_t lds, void* ws, size_t ws_bytes, void* stream) {
  return deig_syrk_f32_ex(X, n, d, ldx, alpha, S, lds, DEIG_SYRK_DEFAULT, ws, ws_bytes, stream);
}

size_t deig_syrk_u8_workspace(int64_t n, int64_t d, int mode) {
  return syrk_u8_workspace_bytes(n, d, mode);
}

int deig_syrk_u8(const uint8_t* X, int64_t n, int64_t d, int64_t ldx, int mode, double alpha,
                 float* S, int64_t lds, double* S64, int64_t lds64, void* ws, size_t ws_bytes,
                 void* stream) {
  g_err[0] = 0;
  return syrk_u8_launch(X, n, d, ldx, mode, alpha, S, lds, S64, lds64, ws, ws_bytes,
                        (hipStream_t)stream);
}

int deig_default_subspace(int64_t d, int k) {
  int64_t p = ((int64_t)k + (k < 16 ? 8 : k / 4) + 15) / 16 * 16;
  if (p > kMaxP) p = kMaxP;
  if (p > d) p = d / 16 * 16;
  if (p < k) p = (k + 15) / 16 * 16;
  return (int)p;
}

size_t deig_topk_workspace(int64_t d, int k, int p) {
  if (p <= 0) p = deig_default_subspace(d, k);
  size_t total = 0;
  carve_solver(nullptr, 0, d, k, p, 0, &total);
  return total;
}

int deig_topk_sym_f32(const float* S, int64_t d, int64_t lds, int k, int p, int max_sweeps,
                      float tol, const float* Q0, int k0, int64_t ldq0, float* V, int64_t ldv,
                      float* evals, int* sweeps_out, float* resid_out, void* ws, size_t ws_bytes,
                      void* stream) {
  g_err[0] = 0;
  if (!S || lds < d || lds % 4 != 0 || !aligned16(S))
    return fail(DEIG_EINVAL, "topk: S must be 16-byte aligned with lds >= d, lds %% 4 == 0");
  Operator op{};
  op.implicit = false;
  op.S = S;
  op.lds = lds;
  return solve(op, d, k, p, max_sweeps, tol, Q0, k0, ldq0, V, ldv, evals, sweeps_out, resid_out,
               ws, ws_bytes, (hipStream_t)stream);
}

size_t deig_projavg_workspace(int64_t d, int64_t mk, int k, int p) {
  if (p <= 0) p = deig_default_subspace(d, k);
  size_t total = 0;
  carve_solver(nullptr, 0, d, k, p, mk, &total);
  return total;
}

int deig_projavg_topk_f32(const float* Wt, int64_t d, int64_t mk, int64_t ldw, float scale, int k,
                          int p, int max_sweeps, float tol, const float* Q0, int k0, int64_t ldq0,
                          float* V, int64_t ldv, float* evals, int* sweeps_out, float* resid_out,
                          void* ws, size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  if (!Wt || mk < 1 || ldw < d || ldw % 4 != 0 || !aligned16(Wt))
    return fail(DEIG_EINVAL, "projavg: Wt must be 16-byte aligned, mk >= 1, ldw >= d, ldw %% 4 == 0");
  Operator op{};
  op.implicit = true;
  op.Wt = Wt;
  op.mk = mk;
  op.ldw = ldw;
  op.scale = scale;
  return solve(op, d, k, p, max_sweeps, tol, Q0, k0, ldq0, V, ldv, evals, sweeps_out, resid_out,
               ws, ws_bytes, (hipStream_t)stream);
}

int deig_sym_power_f32(const float* S, int64_t d, int64_t lds, float* Q, int p, int64_t ldq,
                       float* Y, int64_t ldy, const float* cs, int steps, int algo, void* ws,
                       size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  DEIG_REQUIRE(steps >= 1 && cs && Q, "sym_power: need steps >= 1, cs and Q");
  const bool prepared = (algo & DEIG_SWEEP_PREPARED) != 0;
  const int smode = (algo & DEIG_SWEEP_FAST)      ? kSweepFast
                    : (algo & DEIG_SWEEP_ROUND_Q) ? kSweepRoundQ
                                                  : kSweepExact;
  algo &= ~(DEIG_SWEEP_PREPARED | DEIG_SWEEP_ROUND_Q | DEIG_SWEEP_FAST);
  if (algo != DEIG_SWEEP_AUTO && algo != DEIG_SWEEP_BF16X6)
    return fail(DEIG_EINVAL, "sym_power: algorithm %d has no fused chain (bf16x6 only)", algo);
  hipStream_t st = (hipStream_t)stream;
  if (!prepared) {
    const int rc = sweep_prepare(S, d, lds, p, ws, ws_bytes, st);
    if (rc) return rc;
  }
  SweepStep step{};
  step.kind = 1;
  step.Q = Q;
  step.ldq = ldq;
  step.cs = cs;
  step.lam = cs;  // liveness |cs_j| >= 0 * |cs_0|: every column with cs_j > 0
  step.tau = 0.f;
  step.next_mode = smode;
  for (int i = 0; i < steps; ++i) {
    const int rc = sweep_apply(S, d, lds, Q, p, ldq, Y, ldy, 1.f, ws, ws_bytes, st, smode, &step,
                               i > 0);
    if (rc) return rc;
  }
  return DEIG_OK;
}

size_t deig_sym_apply_workspace(int64_t d, int p, int algo) {
  algo &= ~(DEIG_SWEEP_PREPARED | DEIG_SWEEP_ROUND_Q | DEIG_SWEEP_FAST | DEIG_SWEEP_KERNEL_ONLY);
  if (algo == DEIG_SWEEP_FP32) return skinny_workspace_bytes(d, p, d);
  return sweep_workspace_bytes(d, p);
}

int deig_sym_apply_f32(const float* S, int64_t d, int64_t lds, const float* Q, int p,
                       int64_t ldq, float* Y, int64_t ldy, float alpha, int algo, void* ws,
                       size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  if (algo == DEIG_SWEEP_FP32)
    return skinny_launch(true, S, lds, Q, ldq, Y, ldy, d, p, d, alpha, 0.f,
                         static_cast<float*>(ws), ws_bytes, (hipStream_t)stream);
  const bool prepared = (algo & DEIG_SWEEP_PREPARED) != 0;
  const bool kernel_only = (algo & DEIG_SWEEP_KERNEL_ONLY) != 0;
  const int smode = (algo & DEIG_SWEEP_FAST)      ? kSweepFast
                    : (algo & DEIG_SWEEP_ROUND_Q) ? kSweepRoundQ
                                                  : kSweepExact;
  algo &= ~(DEIG_SWEEP_PREPARED | DEIG_SWEEP_ROUND_Q | DEIG_SWEEP_FAST | DEIG_SWEEP_KERNEL_ONLY);
  if (algo != DEIG_SWEEP_AUTO && algo != DEIG_SWEEP_BF16X6)
    return fail(DEIG_EINVAL, "sym_apply: unknown algorithm %d", algo);
  if (!prepared) {
    const int rc = sweep_prepare(S, d, lds, p, ws, ws_bytes, (hipStream_t)stream);
    if (rc) return rc;
  }
  return sweep_apply(S, d, lds, Q, p, ldq, Y, ldy, alpha, ws, ws_bytes, (hipStream_t)stream,
                     smode, nullptr, kernel_only, kernel_only);
}

size_t deig_oja_workspace(int64_t b, int64_t d, int k) { return oja_workspace_bytes(b, d, k); }

int deig_oja_steps_f32(const float* X, int64_t nb, int64_t b, int64_t d, int64_t ldx, float eta,
                       float* V, int k, int64_t ldv, int orth_every, void* ws, size_t ws_bytes,
                       void* stream) {
  g_err[0] = 0;
  if (!X || !V || !aligned16(X)) return fail(DEIG_EINVAL, "oja: X must be 16-byte aligned");
  return oja_steps_launch(X, nb, b, d, ldx, eta, V, k, ldv, orth_every, ws, ws_bytes,
                          (hipStream_t)stream);
}

int deig_oja_step_f32(const float* Xb, int64_t b, int64_t d, int64_t ldx, float eta, float* V,
                      int k, int64_t ldv, void* ws, size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  if (!Xb || !V || !aligned16(Xb)) return fail(DEIG_EINVAL, "oja: Xb must be 16-byte aligned");
  return oja_launch(Xb, b, d, ldx, eta, V, k, ldv, ws, ws_bytes, (hipStream_t)stream);
}

size_t deig_project_workspace(int64_t n, int64_t d, int k) {
  return project_workspace_bytes(n, d, k);
}

int deig_project_f32(const float* X, int64_t n, int64_t d, int64_t ldx, const float* W, int k,
                     int64_t ldw, float* Y, int64_t ldy, void* ws, size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  return project_launch(X, n, d, ldx, W, k, ldw, Y, ldy, ws, ws_bytes, (hipStream_t)stream);
}

size_t deig_gemm_skinny_workspace(int64_t M, int64_t N, int64_t K) {
  return skinny_workspace_bytes(M, N, K);
}

int deig_gemm_skinny_f32(int trans_a, const float* A, int64_t lda, const float* B, int64_t ldb,
                         float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, float alpha,
                         float beta, void* ws, size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  return skinny_launch(trans_a != 0, A, lda, B, ldb, C, ldc, M, N, K, alpha, beta,
                       static_cast<float*>(ws), ws_bytes, (hipStream_t)stream);
}

}  // extern "C"
