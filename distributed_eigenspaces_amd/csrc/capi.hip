// extern "C" boundary of libdeig.so (declared in include/deig.h) and the host
// drivers of the two eigensolvers.  No device allocation happens here: all
// device memory is caller-provided (PyTorch tensors on the Python side).  No
// process-global mutable state beyond: the error string (thread-local), the per-device
// CU counts (atomics) and a mutex-protected free list of small pinned host blocks the
// solvers read their per-cycle status from (HostStatus); solver behaviour comes from
// the caller's options.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <math.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <tuple>
#include <vector>

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
  static std::atomic<int> cache[64];  // zero-initialised (static storage)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return 256;  // MI355X; only reached by workspace queries without a device
  }
  int v = cache[dev].load(std::memory_order_relaxed);
  if (!v) {
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0) {
      (void)hipGetLastError();
      v = 256;
    }
    cache[dev].store(v, std::memory_order_relaxed);  // same value from every thread
  }
  return v;
}

namespace {

constexpr int kMaxP = 128;
// Block locking (k > kMaxP): each block targets kMaxP - kGuard pairs with kGuard
// guard columns, then locks them and deflates them out of the operator.
constexpr int kGuard = 16;
// Stagnation handling of the solver (see iterate()): a stalled residual counts as
// converged when <= max(kStallAcceptTol * tol, kStallAcceptAbs) - the fp32 floor
// of ||S v - lambda v|| / |lambda_max| is a few 1e-7 up to d = 16384 - and the
// solver gives up after kStallGiveUp Rayleigh-Ritz steps without a 10% gain.
constexpr float kStallAcceptTol = 4.0f;
constexpr float kStallAcceptAbs = 2e-6f;
constexpr int kStallGiveUp = 12;
// Deflation of dominant pairs (see solve()): eigenpairs with theta_j >=
// kDeflateRatio * theta_{k-1} (at most kMaxDeflate of them) are locked, deflated
// out of the operator and the rest iterated again.
constexpr float kDeflateRatio = 64.f;
constexpr int kMaxDeflate = 8;
// Indefinite input: a block whose Ritz values include theta_min < -max(kNegRel *
// scale, kNegTarget * theta_target) restarts the solve on S + sigma I,
// sigma = kShiftGrow * |theta_min| (at most kMaxShifts restarts).
constexpr float kNegRel = 1e-5f;
// Deflation-residue band of the convergence test (cycle_finish): a block whose largest
// |Ritz value| is at most kBandRel * |lambda_max| is judged by its residual against
// |lambda_max| (its own ~0 Ritz values never reach tol).  32 fp32 ulps of the scale:
// the level of deflation residue and fp32 rounding of S, not of small but genuine
// eigenvalues (the band at kNegRel = 1e-5 also took eigenvalues up to 1e-5
// of lambda_max, whose own-relative residual then only reached ~0.1).
constexpr float kBandRel = 32.f * 1.1920929e-7f;
constexpr float kNegTarget = 0.1f;
constexpr double kShiftGrow = 1.1;
constexpr int kMaxShifts = 2;
constexpr double kChebGmax = 1e4;
constexpr int kChebMaxDeg = 16;

struct Opts {
  int sweep_algo = DEIG_SWEEP_BF16X6;
  int rr_every = 0;
  bool cheb = true;
  float cheb_above = -1.f;  // < 0: per solve (Solver::iter_begin)
  bool deflate = true;
  bool deflate_early = true;
  int jcap_sweeps = -1;
  float jcap_above = -1.f;
  float fast_until = 1e-3f;
  float round_until = 1e-4f;
  float half_until = 1e-2f;
  bool debug = false;
};

Opts make_opts(const deig_solver_opts* o) {
  Opts r;
  if (!o) return r;
  r.sweep_algo = o->sweep_algo == DEIG_SWEEP_FP32 ? DEIG_SWEEP_FP32 : DEIG_SWEEP_BF16X6;
  r.rr_every = o->rr_every;
  r.cheb = o->chebyshev != 0;
  r.cheb_above = o->cheb_above;
  r.deflate = o->deflate != 0;
  r.deflate_early = o->deflate_early != 0;
  r.jcap_sweeps = o->jacobi_early_sweeps;
  r.jcap_above = o->jacobi_early_above;
  r.fast_until = o->fast_until;
  r.round_until = o->round_until;
  r.half_until = o->half_until;
  r.debug = o->debug != 0;
  return r;
}

struct Operator {
  bool implicit;
  const void* S;  // explicit: d x d row-major (lds), element type stype
  int stype;
  int64_t lds;
  const float* Wt;  // implicit: scale * Wt^T Wt
  int64_t mk, ldw;
  float scale;
  // applied on top of the base operator (image: folded in by sweep_prepare;
  // plain products: applied after each product): + shift I - Vd diag(lamd) Vd^T
  double shift;
  const float* Vd;
  int64_t ldvd;
  const float* lamd;
  int r;
};

struct SolverWs {
  RRBuffers rr;
  float* Zt;
  float* T;     // d x p: X_{j-1} of the Chebyshev recurrence
  float* Tdef;  // k x p: Vd^T Q of the plain-product deflation
  void* rq;     // partial sums of the final double-precision Rayleigh quotients
  float* slab;
  size_t slab_bytes;
  void* sweep_ws;  // bf16x6 sweep image (explicit S only)
  size_t sweep_bytes;
};

// p: the widest block subspace, kb: the most pairs one block targets (<= p), k:
// all pairs (locked ones are deflated by plain products when there is no image).
SolverWs carve_solver(void* ws, size_t cap, int64_t d, int kb, int k, int p, int64_t mk,
                      bool image, size_t* total) {
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
  w.rr.resid_part = c.take<float>((size_t)rr_update_blocks(d) * kb);
  w.rr.resid = c.take<float>((size_t)kb + 1);
  w.rr.info = c.take<int>(16);
  w.Zt = mk > 0 ? c.take<float>((size_t)mk * p) : nullptr;
  w.T = c.take<float>((size_t)d * p);
  w.Tdef = image ? nullptr : c.take<float>((size_t)k * p);
  w.rq = mk > 0 ? nullptr : c.take<char>(rq_workspace_bytes(d, k));
  size_t sb = skinny_workspace_bytes(2 * p, 2 * p, d);  // Gram
  auto need = [&](int64_t M, int64_t N, int64_t K) {
    const size_t b = skinny_workspace_bytes(M, N, K);
    if (b > sb) sb = b;
  };
  if (mk > 0) {
    need(mk, p, d);  // Wt Q
    need(d, p, mk);  // Wt^T Zt
  } else if (!image) {
    need(d, p, d);  // S Q
  }
  if (!image) {  // plain-product deflation: Vd^T Q and Vd T
    need(k, p, d);
    need(d, p, k);
  }
  w.slab = c.take<float>(sb / sizeof(float) + 4);
  w.slab_bytes = sb;
  w.sweep_ws = nullptr;
  w.sweep_bytes = 0;
  if (image) {
    w.sweep_bytes = sweep_workspace_bytes(d, p);
    w.sweep_ws = c.take<char>(w.sweep_bytes);
  }
  *total = c.off;
  return w;
}

// Y[r][:] += s Q[r][:] (row strides ldy, ldq; p columns) - the shift on plain products.
__global__ __launch_bounds__(256) void axpy_rows_kernel(float* __restrict__ Y, int64_t ldy,
                                                        const float* __restrict__ Q, int64_t ldq,
                                                        int64_t d, int p, float s) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= d * p) return;
  const int64_t r = idx / p;
  const int j = (int)(idx - r * p);
  Y[r * ldy + j] = fmaf(s, Q[r * ldq + j], Y[r * ldy + j]);
}

// T[q][:] *= -lam[q]  (r x p, row stride p).
__global__ __launch_bounds__(256) void neg_scale_rows_kernel(float* __restrict__ T, int r, int p,
                                                             const float* __restrict__ lam) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)r * p) return;
  T[idx] *= -lam[idx / p];
}

// Y = A Q without a sweep image: the fp32 skinny product (explicit S) or the
// implicit projector average Wt^T (Wt Q) (the server), then the shift and the
// deflation of the locked pairs as products with Vd.
int apply_op_plain(const Operator& op, const SolverWs& w, int64_t d, int p, hipStream_t st) {
  float* Q = w.rr.Z;
  float* Y = w.rr.Z + p;
  const int64_t ld = 2 * p;
  int rc;
  if (!op.implicit) {
    rc = skinny_launch(true, static_cast<const float*>(op.S), op.lds, Q, ld, Y, ld, d, p, d, 1.f,
                       0.f, w.slab, w.slab_bytes, st);
  } else {
    rc = skinny_launch(false, op.Wt, op.ldw, Q, ld, w.Zt, p, op.mk, p, d, 1.f, 0.f, w.slab,
                       w.slab_bytes, st);
    if (rc) return rc;
    rc = skinny_launch(true, op.Wt, op.ldw, w.Zt, p, Y, ld, d, p, op.mk, op.scale, 0.f, w.slab,
                       w.slab_bytes, st);
  }
  if (rc) return rc;
  if (op.shift != 0.0) {
    hipLaunchKernelGGL(axpy_rows_kernel, dim3((unsigned)cdiv(d * p, 256)), dim3(256), 0, st, Y, ld,
                       Q, ld, d, p, (float)op.shift);
    DEIG_HIP_CHECK(hipGetLastError());
  }
  if (op.r > 0) {
    DEIG_REQUIRE(op.ldvd % 4 == 0, "solver: deflation needs ldv %% 4 == 0 (ldv=%lld)",
                 (long long)op.ldvd);
    // Tdef = Vd^T Q (Vd column-major = r x d row-major), scaled by -lam, Y += Vd Tdef
    if ((rc = skinny_launch(false, op.Vd, op.ldvd, Q, ld, w.Tdef, p, op.r, p, d, 1.f, 0.f, w.slab,
                            w.slab_bytes, st)))
      return rc;
    hipLaunchKernelGGL(neg_scale_rows_kernel, dim3((unsigned)cdiv((int64_t)op.r * p, 256)),
                       dim3(256), 0, st, w.Tdef, op.r, p, op.lamd);
    DEIG_HIP_CHECK(hipGetLastError());
    if ((rc = skinny_launch(true, op.Vd, op.ldvd, w.Tdef, p, Y, ld, d, p, op.r, 1.f, 1.f, w.slab,
                            w.slab_bytes, st)))
      return rc;
  }
  return DEIG_OK;
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
  if (w.sweep_ws)
    return sweep_apply(Q, d, p, ld, Y, ld, 1.f, w.sweep_ws, w.sweep_bytes, st, smode, step, q_ready);
  int rc = apply_op_plain(op, w, d, p, st);
  if (rc || !step) return rc;
  if (step->kind == 1) return rr_power_launch(w.rr, d, p, step->tau, st);
  return cheb_step_launch(w.rr, w.T, d, p, step->thr, step->a, step->cc, step->gamma, st);
}

// Chebyshev filter plan for the sweeps between two Rayleigh-Ritz steps (host side,
// from the last RR's Ritz values theta_0 >= ... >= theta_{p-1} and residual).
// The operator is PSD here (covariances, projector averages, or an indefinite S
// shifted by the solver): the damped interval is [0, c] with c = theta_{p-1} (the
// block's smallest Ritz value) when the basis has guard columns, else
// min(theta_{p-1}, theta_{k-1} / 2).  Scaled recurrence at gamma = theta_0 (Zhou &
// Saad): X_1 = (s1/e)(A - cc) X_0, X_{j+1} = (2 s_{j+1}/e)(A - cc) X_j - s_j s_{j+1}
// X_{j-1}, s_{j+1} = 1/(2/s1 - s_j).  Degree m: at most kChebMaxDeg, at most what
// the residual still needs at column k's damping rate, and small enough that a
// column's contamination by theta_0's direction grows at most gmax = clamp(1/resid,
// 10, kChebGmax) times (the fp32 Gram of the filtered block must still resolve
// every column); columns whose growth would exceed gmax stay out of the filter
// (threshold thr on theta_j).  Only used once resid <= cheb_above (Solver::iter_begin:
// 1.0 - from the first RR on - for single-block explicit solves since r05, else 1e-2):
// before that plain power steps run.  r04 kept 1e-2 everywhere (r04 A/B,
// profiles/r04k_solver_opts_sweep.log and r04m_*): 0.1
// cut synthetic worker solves 6-16 % (c5 18.0 -> 16.6 ms at the same bars) but the c1
// bench's uncentered byte covariances took 31-37 sweeps instead of 28-29 (c1 8.06 ->
// 7.0 M samples/s: the dominant direction holds an early filter to degree 1), and 0.5
// stalled two k > 128 block-locking cases above the accept floor.
struct ChebPlan {
  int m = 0;
  double cc = 0, e = 1, s1 = 0;
  float thr = 0;
};

bool cheb_plan(const float* lam, int k, int p, float resid, float tol, float above, ChebPlan* pl) {
  if (!(resid <= above) || !(resid > 0)) return false;
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

// Per-cycle solver status (residuals, Ritz values, the small solve's Jacobi flag),
// written by status_kernel straight into pinned, mapped host memory and read after
// the cycle's stream sync: one small launch instead of three device-to-host copies
// into pageable memory (each a blit kernel plus a staging round trip that blocks
// the calling thread; c1: 226 copies per step, profiles/r03s).  Blocks come from a
// process-wide free list (allocated on demand and kept: hipHostFree synchronises
// the device, which would serialise the Slave threads' streams).
struct HostStatus {
  float res[kMaxP + 1];
  float lam[kMaxP];
  int jconv;
};

// blockIdx.x: the problem of a batched launch (buffers at pbt.off, status block pbt.hs).
__global__ __launch_bounds__(256) void status_kernel(const float* __restrict__ resid, int nres,
                                                     const float* __restrict__ lam, int pb,
                                                     const int* __restrict__ info,
                                                     const ProbBatch pbt) {
  const int t = threadIdx.x, prob = blockIdx.x;
  HostStatus* __restrict__ hs = static_cast<HostStatus*>(pbt.hs[prob]);
  if (prob) {
    const int64_t o = pbt.off[prob];
    resid = reinterpret_cast<const float*>(reinterpret_cast<const char*>(resid) + o);
    lam = reinterpret_cast<const float*>(reinterpret_cast<const char*>(lam) + o);
    info = reinterpret_cast<const int*>(reinterpret_cast<const char*>(info) + o);
  }
  if (t < nres) hs->res[t] = resid[t];
  if (t < pb) hs->lam[t] = lam[t];
  if (t == 0) hs->jconv = info[3];
}

class StatusPool {
 public:
  int acquire(HostStatus** out) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!free_.empty()) {
      *out = free_.back();
      free_.pop_back();
      return DEIG_OK;
    }
    void* p = nullptr;
    if (hipHostMalloc(&p, sizeof(HostStatus), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess || !p) {
      (void)hipGetLastError();
      return fail(DEIG_EHIP, "solver: pinned status block allocation failed");
    }
    memset(p, 0, sizeof(HostStatus));
    *out = static_cast<HostStatus*>(p);
    return DEIG_OK;
  }
  void release(HostStatus* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu_);
    free_.push_back(p);
  }
  // deig_shutdown: free the idle blocks while the HIP runtime is alive (blocks in use by
  // a running solver come back through release and stay until the next drain)
  void drain() {
    std::lock_guard<std::mutex> lk(mu_);
    for (HostStatus* p : free_) (void)hipHostFree(p);
    free_.clear();
    (void)hipGetLastError();
  }
  bool empty() {
    std::lock_guard<std::mutex> lk(mu_);
    return free_.empty();
  }

 private:
  std::mutex mu_;
  std::vector<HostStatus*> free_;
};

StatusPool& status_pool() {
  static StatusPool pool;  // C++11 thread-safe initialisation; never destroyed before use ends
  return pool;
}

constexpr int64_t kHalfMinD = 2048;  // smallest d for the one-product early sweeps

struct Solver {
  Operator op;
  Opts o;
  int64_t d;
  int max_sweeps;
  float tol;
  SolverWs w;
  hipStream_t st;
  HostStatus* hs = nullptr;  // pinned: the last RR's status (status_kernel)
  const float* lam_h = nullptr;  // hs->lam: Ritz values of the last RR (descending)
  const float* res_h = nullptr;  // hs->res: per-column residuals (descending Ritz order)
  int jconv_h = 1;               // the last RR's Jacobi converged (rr.hip info[3])
  int it = 0;              // sweeps done (all blocks and restarts)
  float last = 3.4e38f;
  bool converged = false;
  // the iteration in progress (iter_begin .. a cycle_finish that ends it)
  int kc = 0, pb = 0;
  float* Vb = nullptr;
  int64_t ldv = 0;
  float* evb = nullptr;
  bool allow_early = false, early = false;
  int rr_every = 4, jcap_sweeps = 2, jcap = 30, nrr = 0, start = 0, since_best = 0;
  float tau = 0.f, jcap_above = 1e-4f, best = 3.4e38f, cheb_above = 1e-2f;
  // |theta| scale of the whole operator (the first block's Ritz values; 0 until the
  // first block has ended) and the factor that turns the last RR's residuals from
  // "relative to the block's own largest Ritz value" (rr_finish_kernel) into
  // "relative to the operator's scale" - 1 outside the deflation-residue band
  float abs_scale = 0.f, band_f = 1.f;
  bool fuse = false;
  int ncheb_dbg = 0;

  // Pairs a block's dominant-pair deflation would lock (0: none).
  int dominant(int kc_) const {
    if (!(lam_h[kc_ - 1] > 0.f && lam_h[0] >= kDeflateRatio * lam_h[kc_ - 1])) return 0;
    int r = 0;
    while (r < kc_ - 1 && r < kMaxDeflate && lam_h[r] >= kDeflateRatio * lam_h[kc_ - 1]) ++r;
    return r;
  }

  // Subspace iteration for the top kc pairs of the current operator on a pb-column
  // basis (initialised by the caller); the pairs go to Vb / evb (ascending).
  // allow_early: stop as soon as the dominant pairs are converged (early).
  //   A cycle = [filter / power sweeps] + one sweep with a Rayleigh-Ritz step (Gram +
  // small solve + update + residual check): cycle_sweeps (through the Gram),
  // cycle_rr_small, cycle_update (+ the residual copies), a stream sync, then
  // cycle_finish.  The batched driver (solve_batch) runs the small solves of several
  // problems in one launch between cycle_sweeps and cycle_update.
  //   Between two RRs either a Chebyshev filter of planned degree runs (cheb_plan)
  // or, while the residual is above cheb_above, rr_every - 1 plain power steps
  // Q <- A Q on the Ritz vectors of the last RR (same span as subspace iteration;
  // the generalised RR copes with the non-orthonormal basis).  The single-workgroup
  // small solve is the latency-bound part of a cycle, so spacing RRs divides its
  // cost.  Power steps: every 4th sweep is an RR when the basis has >= 16 guard
  // columns beyond k (measured: d=8192 k=64 p=80 6.2 vs 9.0 ms, d=3072 k=16 p=32 1.4
  // vs 1.9 ms); every 2nd without them (d=16384 k=128 p=128: 23 sweeps / 47 ms vs
  // 41 / 54 ms).
  void iter_begin(int kc_, int pb_, float* Vb_, int64_t ldv_, float* evb_, bool allow_early_,
                  bool single_block) {
    kc = kc_;
    pb = pb_;
    Vb = Vb_;
    ldv = ldv_;
    evb = evb_;
    allow_early = allow_early_;
    early = false;
    rr_every = o.rr_every > 0 ? o.rr_every : (pb - kc >= 16 ? 4 : 2);
    tau = rr_every > 1 ? powf(0.1f, 1.0f / (float)(rr_every - 1)) : 0.f;
    // Early Rayleigh-Ritz steps run a capped Jacobi: worker solves (explicit S) 2
    // sweeps while the residual is above 1e-4 (r02s A/B, profiles/r02s_jacobi_cap_ab.log:
    // c1 +8 %, c1g +14 % over 3 above 1e-2, c3 the same time in 16 sweeps instead of
    // 12; 1 sweep fails the bars); the server's implicit projector average
    // (eigenvalues clustered near 1) 3 above 1e-2 (the tighter cap cost config 4's
    // aggregation 2.05 -> 2.65 ms).
    jcap_sweeps = o.jcap_sweeps >= 0 ? o.jcap_sweeps : (op.implicit ? 3 : 2);
    // a basis spanning the whole space (tiny d, k close to d): the first Rayleigh-Ritz
    // step is the exact eigendecomposition - run its Jacobi to convergence
    if (pb >= d) jcap_sweeps = 0;
    jcap_above = o.jcap_above >= 0.f ? o.jcap_above : (op.implicit ? 1e-2f : 1e-4f);
    // The Chebyshev filter from the first Rayleigh-Ritz step on for a single-block
    // solve of an explicit S on a basis without guard columns (p - k < 4: the filter's
    // interval ends at theta_k / 2, which holds from the first RR on), else once resid
    // <= 1e-2 (r05, tools/solver_opts_sweep.py and tools/cheb_policy_ab.py,
    // profiles/r05w_*: config-5 worker 14.5 -> 11.9 ms, the p = k test spectrum 6.87 ->
    // 6.18 ms, same bars; with guard columns the early interval ends at an unconverged
    // guard Ritz value: config-3 shard 3.10 -> 3.05 ms but the spiked d = 3072 test
    // 13 -> 14 sweeps, 0.857 -> 0.884 ms; block locking, k > 128, stalled above the
    // accept floor with the early filter, as in r04; the implicit projector averages
    // are clustered near 1).
    cheb_above = o.cheb_above >= 0.f ? o.cheb_above
                                     : ((single_block && !op.implicit && pb - kc < 4) ? 1.0f : 1e-2f);
    fuse = w.sweep_ws != nullptr;
    best = 3.4e38f;
    since_best = 0;
    nrr = 0;
    start = it;
    last = 3.4e38f;
    converged = false;
  }

  // The cycle's sweeps, planned on the host (plan_cycle) and then enqueued (run_plan,
  // or solve_batch's batched launches across problems).
  struct PlanItem {
    SweepStep step;
    bool has_step;  // a fused basis step follows the product
    int smode;
    bool q_ready;   // this sweep's Q image was written by the previous one
  };
  std::vector<PlanItem> plan;

  // Enqueue the cycle's sweeps and the Gram; *ended: the sweep budget is spent (the
  // iteration is over, nothing was enqueued).
  int cycle_sweeps(bool* ended) {
    plan_cycle(ended);
    if (*ended) return DEIG_OK;
    int rc;
    for (const PlanItem& pi : plan)
      if ((rc = apply_op(op, w, d, pb, st, pi.smode, pi.has_step ? &pi.step : nullptr, pi.q_ready)))
        return rc;
    return gram(st);
  }

  int gram(hipStream_t s) {
    return skinny_launch(true, w.rr.Z, 2 * pb, w.rr.Z, 2 * pb, w.rr.C, 2 * pb, 2 * pb, 2 * pb, d, 1.f,
                         0.f, w.slab, w.slab_bytes, s);
  }

  void plan_cycle(bool* ended) {
    plan.clear();
    *ended = !(it - start < max_sweeps);
    if (*ended) return;
    const int budget = max_sweeps - (it - start);
    // Sweep precision by residual: early sweeps (above fast_until) take S as its
    // two leading bf16 pieces too - three products, no split in the sweep, ~2^-16
    // relative (sweep.hip sweep_products SP = 2), 100x below the residual there;
    // then Q rounded to two pieces (five products) down to round_until; the
    // closing sweeps exact (the rounding puts ~4e-6 relative noise into the basis
    // each sweep: a floor under the residual).
    // One-product sweeps (~2^-9) while the residual is above half_until, from
    // d = 2048 on: there the sweep streams S from HBM and the mode halves its bytes
    // (c5 worker solve 8.3 -> 6.9 ms); below it the sweep is latency-bound, and two
    // small-d edge cases (k = 97 of d = 100, k = 200 rank-deficient at d = 512) lost
    // convergence with it.
    const bool half_ok = o.half_until > 0.f && d >= kHalfMinD;
    const int smode = (half_ok && last > fmaxf(o.half_until, tol))                ? kSweepHalf
                      : (o.fast_until > 0.f && last > fmaxf(o.fast_until, tol)) ? kSweepFast
                      : last > fmaxf(o.round_until, tol)                      ? kSweepRoundQ
                                                                              : kSweepExact;
    ChebPlan cp;
    const bool cheb = o.cheb && nrr > 0 && cheb_plan(lam_h, kc, pb, last, tol, cheb_above, &cp);
    int nstep = 0;
    ncheb_dbg = 0;
    SweepStep step{};
    step.Q = w.rr.Z;
    step.ldq = 2 * pb;
    step.T = w.T;
    step.cs = w.rr.cs;
    step.lam = w.rr.lam;
    step.next_mode = smode;
    if (cheb) {
      // degree j: apply A to X_j, then X_{j+1} from X_j, A X_j and X_{j-1}
      const int m = std::min(cp.m, budget - 1);
      double s_prev = cp.s1;
      for (int j = 0; j < m; ++j, ++it, ++nstep) {
        double alpha, gamma;
        if (j == 0) {
          alpha = cp.s1 / cp.e;
          gamma = 0.0;
        } else {
          const double s_next = 1.0 / (2.0 / cp.s1 - s_prev);
          alpha = 2.0 * s_next / cp.e;
          gamma = s_prev * s_next;
          s_prev = s_next;
        }
        step.kind = 2;
        step.thr = cp.thr;
        step.a = (float)alpha;
        step.cc = (float)cp.cc;
        step.gamma = (float)gamma;
        plan.push_back({step, true, smode, fuse && nstep > 0});
      }
      ncheb_dbg = m;
    } else if (nrr > 0) {
      const int npow = std::min(rr_every - 1, budget - 1);
      // power steps on the live Ritz columns of the last RR (Q_j <- Y_j / ||Y w_j||)
      step.kind = 1;
      step.tau = tau;
      for (int j = 0; j < npow; ++j, ++it, ++nstep) plan.push_back({step, true, smode, fuse && nstep > 0});
    }
    plan.push_back({step, false, smode, fuse && nstep > 0});
    ++it;
    // The next basis Y W spans span(Y) for any invertible W, so subspace progress
    // does not need converged Ritz vectors; the residual of approximate pairs only
    // over-states the error (no false convergence).
    jcap = (jcap_sweeps > 0 && last > jcap_above) ? jcap_sweeps : 30;
  }

  int cycle_rr_small() { return rr_small_launch(w.rr, pb, st, jcap); }

  // Ritz vectors / residuals and their copies to the host (read after a sync).
  int cycle_update() {
    int rc;
    if ((rc = rr_update_launch(w.rr, d, pb, kc, Vb, ldv, evb, st))) return rc;
    ProbBatch one = one_problem();
    one.hs[0] = hs;
    hipLaunchKernelGGL(status_kernel, dim3(1), dim3(256), 0, st, w.rr.resid, kc + 1, w.rr.lam, pb,
                       w.rr.info, one);
    DEIG_HIP_CHECK(hipGetLastError());
    return DEIG_OK;
  }

  // After the sync: *done = the iteration is over (converged, early exit or stalled).
  int cycle_finish(bool* done) {
    *done = false;
    jconv_h = jcap < 30 ? hs->jconv : 1;
    // A block in the deflation-residue band - every Ritz value ~0 next to the
    // operator's scale: a rank-deficient S with k above its rank, or k close to d,
    // after the locked pairs were deflated to ~0 - has residuals relative to its own
    // ~0 Ritz values, which never fall below tol.  It is judged by the documented
    // criterion instead (include/deig.h): ||S v - lambda v|| / |lambda_max(S)|.
    band_f = 1.f;
    if (abs_scale > 0.f) {
      const float blk = fmaxf(fabsf(lam_h[0]), 1e-30f);
      if (blk <= kBandRel * abs_scale) band_f = blk / abs_scale;
    }
    last = res_h[kc] * band_f;
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
    if (o.debug) {
      int inf[9] = {0};
      DEIG_HIP_CHECK(hipMemcpy(inf, w.rr.info, sizeof(inf), hipMemcpyDeviceToHost));
      fprintf(stderr, "[deig] d=%lld k=%d p=%d sweep %d resid %.3e cheb_deg %d chol_floor %d "
              "jacobi_sweeps %d rotations %d small-solve us: chol %.1f linv %.1f congr %.1f "
              "jacobi %.1f tail %.1f\n",
              (long long)d, kc, pb, it, last, ncheb_dbg, inf[0], inf[1], inf[2], inf[4] * 0.01,
              (inf[5] - inf[4]) * 0.01, (inf[6] - inf[5]) * 0.01, (inf[7] - inf[6]) * 0.01,
              (inf[8] - inf[7]) * 0.01);
    }
    if (!(last == last) || last > 3.0e38f)  // NaN / Inf
      return fail(DEIG_EINVAL, "solver: non-finite residual (input contains NaN/Inf?)");
    if (!exact_rr) return DEIG_OK;
    if (last <= tol) {
      converged = true;
      *done = true;
      return DEIG_OK;
    }
    if (allow_early) {
      const int r = dominant(kc);
      bool ok = r >= 1;
      for (int j = 0; j < r && ok; ++j) ok = res_h[j] * band_f <= tol;
      if (ok) {
        early = true;
        *done = true;
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
    } else if (++since_best >= 4 && it - start >= 8) {
      if (last <= fmaxf(kStallAcceptTol * tol, kStallAcceptAbs)) {
        converged = true;
        *done = true;
        return DEIG_OK;
      }
      if (since_best >= kStallGiveUp) *done = true;
    }
    return DEIG_OK;
  }

  // (Re)build the sweep image of the current operator (explicit S only).
  int prepare(int pb_) {
    if (!w.sweep_ws) return DEIG_OK;
    return sweep_prepare(op.S, op.stype, d, op.lds, pb_, w.sweep_ws, w.sweep_bytes, st, op.Vd,
                         op.ldvd, op.lamd, op.r, op.shift);
  }
};

int default_subspace(int64_t d, int k) {
  if (k > kMaxP) return (int)std::min<int64_t>(kMaxP, d / 16 * 16);
  int64_t p = ((int64_t)k + (k < 16 ? 8 : k / 4) + 15) / 16 * 16;
  if (p > kMaxP) p = kMaxP;
  if (p > d) p = d / 16 * 16;
  if (p < k) p = (k + 15) / 16 * 16;
  return (int)p;
}

// Block structure: pairs per full block and the widest block subspace.
void block_shape(int64_t d, int k, int p_in, int* p_blk, int* kb) {
  if (k <= kMaxP) {
    *p_blk = p_in > 0 ? p_in : default_subspace(d, k);
    *kb = k;
  } else {
    *p_blk = p_in > 0 ? p_in : default_subspace(d, k);
    *kb = *p_blk - kGuard;
  }
}

// Any d (?syevr's contract, distributed.py:29): an explicit S whose dimension the
// kernels cannot take as it is - d % 4 != 0, d < 16, or a subspace wider than d (k
// close to a small d) - is staged in the workspace as a zero-padded dp x dp copy, and
// the solver runs on that.  Its padding directions must never outrank S's own
// eigenpairs, which a zero padding (eigenvalue 0) would for an indefinite S whose
// top k reach below 0:
//  * basis narrower than d: every start basis has zero rows >= d (rr_init's `valid`),
//    and S Q, the shift, the deflation and Rayleigh-Ritz all keep zero rows zero, so
//    the padding never enters the iteration;
//  * basis as wide as the padded space (pb > d, tiny d): the padding diagonal is set
//    to -(2R) - tiny, R = max_i sum_j |S_ij| >= the spectral radius, strictly below
//    S's spectrum (the solver then sees an indefinite operator and shifts it).
// V is computed in the padded space and its first d rows copied out.
struct Dims {
  int64_t dp;   // the solver's dimension
  int pb, kb;   // widest block subspace, pairs per block
  bool staged;  // S copied into a padded dp x dp image in the workspace
  bool fill;    // the padding diagonal set below S's spectrum
};

Dims solver_dims(int64_t d, int k, int p, bool implicit) {
  Dims m{};
  m.dp = d;
  if (!implicit) {
    int64_t dp = std::max<int64_t>(16, cdiv(d, 4) * 4);
    int pb, kb;
    block_shape(dp, k, p, &pb, &kb);
    if (pb > dp) dp = pb;
    m.dp = dp;
  }
  block_shape(m.dp, k, p, &m.pb, &m.kb);
  m.staged = m.dp != d;
  m.fill = m.staged && m.pb > d;
  return m;
}

struct Stage {
  void* S = nullptr;  // dp x dp, element type of the input
  float* V = nullptr; // dp x k column-major
  float* Q0 = nullptr;  // dp x pb column-major (warm start)
};

Stage carve_stage(Carve& c, const Dims& m, int k, int stype) {
  Stage g;
  if (!m.staged) return g;
  const size_t es = stype == DEIG_F64 ? sizeof(double) : sizeof(float);
  g.S = c.take<char>((size_t)(m.dp * m.dp) * es);
  g.V = c.take<float>((size_t)m.dp * k);
  g.Q0 = c.take<float>((size_t)m.dp * m.pb);
  c.off = align_up(c.off, 256);
  return g;
}

template <typename T>
__global__ __launch_bounds__(256) void stage_pad_kernel(const T* __restrict__ S, int64_t lds, int64_t d,
                                                        T* __restrict__ Sp, int64_t dp) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= dp * dp) return;
  const int64_t i = idx / dp, j = idx - i * dp;
  Sp[idx] = (i < d && j < d) ? S[i * lds + j] : T(0);
}

// One workgroup (only for d < pb <= kMaxP): R = max_i sum_j |S_ij| in double, then the
// padding diagonal entries dp > i >= d set to -(2R) - 1e-30.
template <typename T>
__global__ __launch_bounds__(256) void stage_fill_kernel(T* __restrict__ Sp, int64_t dp, int64_t d) {
  __shared__ double red[256];
  const int t = threadIdx.x;
  double m = 0.0;
  for (int64_t i = t; i < d; i += 256) {
    double s = 0.0;
    for (int64_t j = 0; j < d; ++j) s += fabs((double)Sp[i * dp + j]);
    m = fmax(m, s);
  }
  red[t] = m;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (t < w) red[t] = fmax(red[t], red[t + w]);
    __syncthreads();
  }
  const double v = -(2.0 * red[0]) - 1e-30;
  for (int64_t i = d + t; i < dp; i += 256) Sp[i * dp + i] = (T)v;
}

// dst[r + j ldd] = r < rows_src ? src[r + j lds] : 0 for r < rows_dst, j < ncol.
__global__ __launch_bounds__(256) void copy_cols_kernel(const float* __restrict__ src, int64_t lds,
                                                        int64_t rows_src, float* __restrict__ dst,
                                                        int64_t ldd, int64_t rows_dst, int ncol) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows_dst * ncol) return;
  const int64_t j = idx / rows_dst, r = idx - j * rows_dst;
  dst[r + j * ldd] = r < rows_src ? src[r + j * lds] : 0.f;
}

int copy_cols(const float* src, int64_t lds, int64_t rows_src, float* dst, int64_t ldd,
              int64_t rows_dst, int ncol, hipStream_t st) {
  hipLaunchKernelGGL(copy_cols_kernel, dim3((unsigned)cdiv(rows_dst * ncol, 256)), dim3(256), 0, st,
                     src, lds, rows_src, dst, ldd, rows_dst, ncol);
  DEIG_HIP_CHECK(hipGetLastError());
  return DEIG_OK;
}

template <typename T>
int stage_matrix(const void* S, int64_t lds, int64_t d, void* Sp, const Dims& m, hipStream_t st) {
  hipLaunchKernelGGL(stage_pad_kernel<T>, dim3((unsigned)cdiv(m.dp * m.dp, 256)), dim3(256), 0, st,
                     static_cast<const T*>(S), lds, d, static_cast<T*>(Sp), m.dp);
  DEIG_HIP_CHECK(hipGetLastError());
  if (m.fill) {
    hipLaunchKernelGGL(stage_fill_kernel<T>, dim3(1), dim3(256), 0, st, static_cast<T*>(Sp), m.dp, d);
    DEIG_HIP_CHECK(hipGetLastError());
  }
  return DEIG_OK;
}

// Top-k eigenpairs (ascending) of the operator.  Blocks of at most kb pairs are
// solved top-down; each block's converged pairs are LOCKED at the end of V and
// deflated out of the operator for the blocks below (k > 128 = kMaxP: the Ritz
// problem of one workgroup holds at most 128 columns).  Within a block, dominant
// pairs (theta_j >= 64 theta_k, an uncentered covariance's mean direction) are
// locked first and the rest iterated again on the deflated operator: every fp32
// product S q otherwise loses log2(theta_0 / theta_k) bits of the small directions
// to cancellation.  Deflated images are formed in double (sweep_prepare_kernel).
// A block whose Ritz values show a large negative eigenvalue (S indefinite: the
// filter and power steps favour large |lambda|) restarts the solve on S + sigma I.
//   Written as a state machine so that several independent problems can advance in
// lockstep (solve_batch): BLOCK (set up the next block: image, start basis) ->
// CYCLE (Solver cycles until the iteration ends) -> end_block (lock / redo /
// restart / next block) ... -> FINAL (eigenvalues) -> DONE.
struct SolveSM {
  enum State { BLOCK, CYCLE, FINAL, DONE };
  Operator op0;
  int64_t d = 0;
  int k = 0, pb0 = 0, kb = 0, k0 = 0;
  const float* Q0 = nullptr;
  int64_t ldq0 = 0;
  float* V = nullptr;
  int64_t ldv = 0;
  float* evals = nullptr;
  // staging (solver_dims): the caller's dimension / V, and the rows >= valid of every
  // start basis that are zero (-1: none)
  int64_t d_user = 0;
  float* V_user = nullptr;
  int64_t ldv_user = 0;
  bool staged = false;
  int64_t valid = -1;
  Solver sv;
  bool can_deflate = false;
  double shift = 0.0;
  float scale = 0.f;  // |theta| scale of the operator (first block's Ritz values)
  bool all_conv = true;
  float worst = 0.f;
  int attempt = 0;
  int locked = 0;     // pairs locked at V columns [k - locked, k)
  bool redo = false;  // re-iterate the rest of a block after locking its dominant pairs
  int warm = 0;       // redo: columns of the block computed before (just below locked)
  int kc = 0, pb = 0;
  float* Vb = nullptr;
  float* evb = nullptr;
  State state = BLOCK;
  int rc = DEIG_OK;

  SolveSM() = default;
  SolveSM(const SolveSM&) = delete;
  SolveSM& operator=(const SolveSM&) = delete;
  ~SolveSM() { status_pool().release(sv.hs); }

  int init(const Operator& op_in, int64_t d_, int k_, int p, int max_sweeps, float tol, const float* Q0_,
           int k0_, int64_t ldq0_, float* V_, int64_t ldv_, float* evals_, const Opts& o, void* ws,
           size_t ws_bytes, hipStream_t st) {
    Operator op = op_in;
    d_user = d_;
    k = k_;
    DEIG_REQUIRE(d_ >= 1, "solver: d=%lld must be >= 1", (long long)d_);
    DEIG_REQUIRE(k >= 1 && k <= d_, "solver: need 1 <= k <= d (k=%d, d=%lld)", k, (long long)d_);
    if (op.implicit)
      DEIG_REQUIRE(d_ >= 16 && d_ % 4 == 0, "solver: d=%lld must be >= 16 and a multiple of 4",
                   (long long)d_);
    DEIG_REQUIRE(V_ && evals_ && ldv_ >= d_, "solver: bad V / evals / ldv");
    DEIG_REQUIRE(k0_ >= 0 && (k0_ == 0 || (Q0_ && ldq0_ >= d_)), "solver: bad warm start");
    const Dims dm = solver_dims(d_, k, p, op.implicit);
    d = dm.dp;
    staged = dm.staged;
    valid = (dm.staged && !dm.fill) ? d_ : -1;
    Carve cs(ws, ws_bytes);
    const Stage stg = carve_stage(cs, dm, k, op.stype);
    if (ws && cs.off > ws_bytes)
      return fail(DEIG_EWORKSPACE, "solver: workspace %zu bytes < staging %zu", ws_bytes, cs.off);
    void* ws_solver = ws ? static_cast<char*>(ws) + cs.off : nullptr;
    const size_t ws_solver_bytes = ws ? ws_bytes - cs.off : 0;
    if (staged && ws) {
      int r = op.stype == DEIG_F64 ? stage_matrix<double>(op.S, op.lds, d_, stg.S, dm, st)
                                   : stage_matrix<float>(op.S, op.lds, d_, stg.S, dm, st);
      if (r) return r;
      op.S = stg.S;
      op.lds = d;
      if (k0_ > 0) {
        if ((r = copy_cols(Q0_, ldq0_, d_, stg.Q0, d, d, std::min(k0_, dm.pb), st))) return r;
        Q0_ = stg.Q0;
        ldq0_ = d;
      }
      V_user = V_;
      ldv_user = ldv_;
      V_ = stg.V;
      ldv_ = d;
    }
    pb0 = dm.pb;
    kb = dm.kb;
    if (k <= kMaxP)
      DEIG_REQUIRE(pb0 % 16 == 0 && pb0 >= k && pb0 <= kMaxP && pb0 <= d,
                   "solver: subspace p=%d must be a multiple of 16 with k <= p <= min(128, d)", pb0);
    else
      DEIG_REQUIRE(pb0 % 16 == 0 && pb0 >= 2 * kGuard && pb0 <= kMaxP && pb0 <= d,
                   "solver: k=%d > 128 needs a block subspace p in {32, ..., 128} (p=%d)", k, pb0);
    DEIG_REQUIRE(max_sweeps >= 1, "solver: max_sweeps must be >= 1");
    DEIG_REQUIRE(k0_ <= pb0, "solver: warm start k0=%d wider than the subspace p=%d", k0_, pb0);
    const bool image = !op.implicit && o.sweep_algo != DEIG_SWEEP_FP32;
    DEIG_REQUIRE(image || op.implicit || op.stype == DEIG_F32,
                 "solver: a float64 S needs the bf16x6 sweep (DEIG_SWEEP_AUTO)");
    size_t total = 0;
    if (!sv.hs) {
      int r = status_pool().acquire(&sv.hs);
      if (r) return r;
      sv.lam_h = sv.hs->lam;
      sv.res_h = sv.hs->res;
    }
    sv.w = carve_solver(ws_solver, ws_solver_bytes, d, kb, k, pb0, op.implicit ? op.mk : 0, image, &total);
    if (!ws || total > ws_solver_bytes)
      return fail(DEIG_EWORKSPACE, "solver: workspace %zu bytes < required %zu", ws_bytes, total + cs.off);
    op0 = op;
    sv.op = op;
    sv.o = o;
    sv.d = d;
    sv.max_sweeps = max_sweeps;
    sv.tol = tol;
    sv.st = st;
    Q0 = Q0_;
    k0 = k0_;
    ldq0 = ldq0_;
    V = V_;
    ldv = ldv_;
    evals = evals_;
    can_deflate = o.deflate && !op.implicit && k >= 2;
    state = BLOCK;
    return DEIG_OK;
  }

  // BLOCK: the next block's operator, sweep image and start basis; -> CYCLE or FINAL.
  int start_block() {
    if (locked >= k) {
      state = FINAL;
      return DEIG_OK;
    }
    const int rem = k - locked;
    kc = rem <= kb ? rem : kb;
    // the last block of k > 128 pairs: the default subspace for its size
    pb = (rem <= kb && k > kMaxP) ? std::min(default_subspace(d, kc), pb0) : pb0;
    Vb = V + (int64_t)(k - locked - kc) * ldv;
    evb = evals + (k - locked - kc);
    sv.op.shift = shift;
    sv.op.r = locked;
    sv.op.Vd = locked ? V + (int64_t)(k - locked) * ldv : nullptr;
    sv.op.ldvd = ldv;
    sv.op.lamd = locked ? evals + (k - locked) : nullptr;
    int r;
    if ((r = sv.prepare(pb))) return r;
    if (redo) {  // warm start: the block's columns below the dominant pairs
      r = rr_init_launch(sv.w.rr.Z, d, pb, V + (int64_t)(k - locked - warm) * ldv, warm, ldv,
                         0x5eed5eefull + locked, sv.st, valid);
    } else if (locked == 0 && k <= kMaxP) {
      r = rr_init_launch(sv.w.rr.Z, d, pb, Q0, k0, ldq0, 0x5eed5eedull, sv.st, valid);
    } else {
      r = rr_init_launch(sv.w.rr.Z, d, pb, nullptr, 0, 0, 0x5eed5eedull + locked, sv.st, valid);
    }
    if (r) return r;
    sv.iter_begin(kc, pb, Vb, ldv, evb, can_deflate && sv.o.deflate_early && !redo, k <= kMaxP);
    state = CYCLE;
    return DEIG_OK;
  }

  // The block's iteration has ended: lock / redo / restart / next block.
  int end_block() {
    int r;
    if (locked > 0) {
      if ((r = deflate_orth_launch(Vb, ldv, d, kc, locked, sv.st))) return r;
      // A block whose Ritz values sit in the deflation-residue band (k close to d, or
      // a rank-deficient operator with k > rank: the locked pairs, deflated to ~0,
      // compete with S's own ~0 eigenvalues) can hold columns that were mostly locked
      // directions: their projected remainders are valid near-null vectors, but not
      // orthogonal to each other - re-orthonormalise the block (rare path).
      bool band = false;
      for (int j = 0; j < kc; ++j) band |= fabsf(sv.lam_h[j]) <= kNegRel * scale;
      if (band && (r = block_mgs_launch(Vb, ldv, d, kc, sv.st))) return r;
    }
    if (locked == 0 && attempt == 0) scale = fmaxf(fabsf(sv.lam_h[0]), fabsf(sv.lam_h[pb - 1]));
    sv.abs_scale = scale;
    // Indefinite S: the most negative Ritz value of the block against the block's
    // target (and the operator's scale - deflation residue is ~1e-7 of it).
    const float tmin = sv.lam_h[pb - 1];
    // (a basis spanning the whole space needs no shift: its Rayleigh-Ritz step is exact,
    // no power or filter step ever ranked |lambda|)
    if (!op0.implicit && attempt < kMaxShifts && pb < d &&
        tmin < -fmaxf(kNegRel * scale, kNegTarget * fmaxf(sv.lam_h[kc - 1], 0.f))) {
      shift = kShiftGrow * (shift - (double)tmin);  // |theta_min| of the shifted op
      if (sv.o.debug)
        fprintf(stderr, "[deig] negative Ritz value %.4e: restarting on S + %.4e I\n", tmin, shift);
      ++attempt;
      all_conv = true;
      worst = 0.f;
      locked = 0;
      redo = false;
      warm = 0;
      state = BLOCK;
      return DEIG_OK;
    }
    const int nd = (can_deflate && !redo && (sv.converged || sv.early)) ? sv.dominant(kc) : 0;
    if (sv.o.debug && nd)
      fprintf(stderr, "[deig] locking %d dominant pair(s)%s at sweep %d\n", nd,
              sv.early ? " (early)" : "", sv.it);
    if (nd >= 1 && nd < kc) {
      locked += nd;  // the rest of the block is iterated again (warm) below them
      warm = kc - nd;
      redo = true;
      state = BLOCK;
      return DEIG_OK;
    }
    worst = fmaxf(worst, sv.last);
    if (!sv.converged) all_conv = false;
    locked += kc;
    redo = false;
    state = BLOCK;
    return DEIG_OK;
  }

  // FINAL: eigenvalues - double-precision Rayleigh quotients on S itself (explicit
  // S; they need no unshift), the projector average's fp32 Ritz values unshifted.
  int finalize() {
    int r = DEIG_OK;
    if (!op0.implicit)
      r = rq_launch(op0.S, op0.stype, d, op0.lds, V, ldv, k, evals, sv.w.rq, sv.st);
    else if (shift != 0.0)
      r = unshift_launch(evals, k, shift, sv.st);
    if (!r && staged) r = copy_cols(V, ldv, d, V_user, ldv_user, d_user, k, sv.st);
    state = DONE;
    return r;
  }

  // Advance through the non-cycling states until CYCLE or DONE.
  int settle() {
    int r;
    while (state == BLOCK || state == FINAL) {
      if (state == BLOCK) {
        if ((r = start_block())) return r;
      } else if ((r = finalize())) {
        return r;
      }
    }
    return DEIG_OK;
  }

  int outcome(int* sweeps_out, float* resid_out) const {
    if (sweeps_out) *sweeps_out = sv.it;
    if (resid_out) *resid_out = rc ? sv.last : worst;
    if (rc) return rc;
    if (!all_conv)
      return fail(DEIG_NOT_CONVERGED, "solver: residual %g > tol %g after %d sweeps%s", worst,
                  sv.tol, sv.it, " (eigengap at k too small for the sweep budget, or stalled)");
    return DEIG_OK;
  }
};

int solve(const Operator& op0, int64_t d, int k, int p, int max_sweeps, float tol, const float* Q0,
          int k0, int64_t ldq0, float* V, int64_t ldv, float* evals, int* sweeps_out,
          float* resid_out, const Opts& o, void* ws, size_t ws_bytes, hipStream_t st) {
  SolveSM sm;
  int rc = sm.init(op0, d, k, p, max_sweeps, tol, Q0, k0, ldq0, V, ldv, evals, o, ws, ws_bytes, st);
  if (rc) return rc;
  while (!rc && sm.state != SolveSM::DONE) {
    if ((rc = sm.settle()) || sm.state == SolveSM::DONE) break;
    bool ended = false, done = false;
    if ((rc = sm.sv.cycle_sweeps(&ended))) break;
    if (ended) {
      rc = sm.end_block();
      continue;
    }
    if ((rc = sm.sv.cycle_rr_small()) || (rc = sm.sv.cycle_update())) break;
    if (hipStreamSynchronize(st) != hipSuccess) {
      rc = fail(DEIG_EHIP, "solver: stream synchronisation failed");
      break;
    }
    if ((rc = sm.sv.cycle_finish(&done))) break;
    if (done) rc = sm.end_block();
  }
  sm.rc = rc;
  return sm.outcome(sweeps_out, resid_out);
}

// Two solvers whose workspaces are carved alike (every buffer at the same offset
// *off from A's): one batched launch can cover both.
bool same_layout(const SolverWs& a, const SolverWs& b, int64_t* off) {
  auto dl = [](const void* y, const void* x) {
    return (int64_t)(reinterpret_cast<uintptr_t>(y) - reinterpret_cast<uintptr_t>(x));
  };
  const int64_t o = dl(b.rr.Z, a.rr.Z);
  *off = o;
  const void* pa[] = {a.rr.C, a.rr.Linv, a.rr.Wtmp, a.rr.W, a.rr.lam, a.rr.cs, a.rr.qs,
                      a.rr.resid_part, a.rr.resid, a.rr.info, a.Zt, a.T, a.Tdef, a.rq, a.slab,
                      a.sweep_ws};
  const void* pb[] = {b.rr.C, b.rr.Linv, b.rr.Wtmp, b.rr.W, b.rr.lam, b.rr.cs, b.rr.qs,
                      b.rr.resid_part, b.rr.resid, b.rr.info, b.Zt, b.T, b.Tdef, b.rq, b.slab,
                      b.sweep_ws};
  for (size_t i = 0; i < sizeof(pa) / sizeof(pa[0]); ++i) {
    if (!pa[i] != !pb[i]) return false;
    if (pa[i] && dl(pb[i], pa[i]) != o) return false;
  }
  return a.slab_bytes == b.slab_bytes && a.sweep_bytes == b.sweep_bytes;
}

// W independent explicit-S problems (same d, k, p) advanced in lockstep by one host
// thread on one stream.  Each round: every problem is brought to its next cycle
// (block set-up, locking, restarts: its own launches) and plans that cycle's sweeps
// (Solver::plan_cycle); then the cycle of all of them is enqueued as batched launches
// - the j-th sweep of every plan in one launch per kernel (sweep.hip SweepBatch: c1's
// 8 problems at d = 3072 each filled only 144 CUs), one Gram launch, the small
// solves in one launch (one workgroup each), one update and one status launch - and
// ONE stream sync precedes every problem's host decision (cycle_finish).  Problems
// are grouped per launch by shape and mode (a block of k > 128 pairs may be
// narrower, a plan shorter); a problem that is done drops out.  r03 ran one host
// thread and stream per problem and met only at the small solves: 8 x 29 sweeps of
// 144 blocks contending for the queues, ~15 small launches per problem and round,
// and a barrier, a sync and a thread wake-up per problem and round (profiles/r04e).
// Results are those of W separate solve() calls (same kernels, split-K slicing and
// decisions; tested bit for bit).
int solve_batch(int W, const Operator* ops, int64_t d, int k, int p, int max_sweeps, float tol,
                float* const* V, int64_t ldv, float* const* evals, int* sweeps_out, float* resid_out,
                int* status_out, const Opts& o, char* ws, size_t ws_each, hipStream_t st) {
  DEIG_REQUIRE(W >= 1 && W <= 1024, "solve_batch: W=%d out of range", W);
  // Two interleaved groups (r06): problems i % 2 == 0 on the caller's stream, the others
  // on a second stream, each group's rounds enqueued right after the host has finished
  // the group's previous round.  While one group's small Rayleigh-Ritz solves run (one
  // workgroup per problem) or the host works through its status, the other group's
  // sweeps fill the GPU.  Every problem's launches are the same as in one group, so the
  // results are too (bit for bit).
  // (d >= 2048: below that the per-launch cost outweighs the overlap - config-1 gray
  // shards, d = 1024, measured 8 % slower with two groups)
#if defined(DEIG_AB_BATCH_ONE_GROUP)
  constexpr int kGroups = 1;
#elif defined(DEIG_AB_BATCH_GROUPS)
  constexpr int kGroups = DEIG_AB_BATCH_GROUPS;
#else
  constexpr int kGroups = 2;
#endif
  constexpr int kMaxGroups = 4;
  static_assert(kGroups >= 1 && kGroups <= kMaxGroups, "stream groups");
  const int NG = d >= 2048 ? std::min(kGroups, W) : 1;
  hipStream_t gs[kMaxGroups] = {st, nullptr, nullptr, nullptr};
  hipEvent_t ev = nullptr;
  struct Cleanup {
    hipStream_t* s;
    hipEvent_t& e;
    ~Cleanup() {
      if (e) (void)hipEventDestroy(e);
      for (int g = 1; g < kMaxGroups; ++g)
        if (s[g]) (void)hipStreamDestroy(s[g]);
    }
  } cleanup{gs, ev};
  if (NG > 1) {
    DEIG_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    DEIG_HIP_CHECK(hipEventRecord(ev, st));  // the operators were written on st
    for (int g = 1; g < NG; ++g) {
      DEIG_HIP_CHECK(hipStreamCreateWithFlags(&gs[g], hipStreamNonBlocking));
      DEIG_HIP_CHECK(hipStreamWaitEvent(gs[g], ev, 0));
    }
  }
  // the caller's stream waits for the other groups' launches (before any return)
  auto join = [&]() -> int {
    for (int g = 1; g < NG; ++g) {
      const hipError_t e1 = hipEventRecord(ev, gs[g]);
      const hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(st, ev, 0) : e1;
      if (e2 != hipSuccess) return fail(DEIG_EHIP, "solve_batch: joining a group's stream failed");
    }
    return DEIG_OK;
  };
  std::vector<SolveSM> sm(W);
  int rc = DEIG_OK;
  for (int i = 0; i < W && !rc; ++i)
    rc = sm[i].init(ops[i], d, k, p, max_sweeps, tol, nullptr, 0, 0, V[i], ldv, evals[i], o,
                    ws + (size_t)i * ws_each, ws_each, gs[i % NG]);
  if (rc) {
    (void)join();
    return rc;
  }
  std::vector<int> grp;
  std::vector<char> taken;
  // Launch groups: up to kMaxProbBatch problems of `mem` that agree on key and are
  // laid out alike; f(grp, batch) enqueues one group.
  auto groups = [&](const std::vector<int>& mem, auto key, auto f) {
    taken.assign(mem.size(), 0);
    for (size_t a = 0; a < mem.size(); ++a) {
      if (taken[a]) continue;
      ProbBatch b = one_problem();
      grp.assign(1, mem[a]);
      taken[a] = 1;
      const auto ka = key(mem[a]);
      for (size_t c = a + 1; c < mem.size() && b.n < kMaxProbBatch; ++c) {
        int64_t off = 0;
        if (taken[c] || !(key(mem[c]) == ka) || !same_layout(sm[mem[a]].sv.w, sm[mem[c]].sv.w, &off))
          continue;
        taken[c] = 1;
        b.off[b.n++] = off;
        grp.push_back(mem[c]);
      }
      if (int r = f(grp, b)) return r;
    }
    return (int)DEIG_OK;
  };
  std::vector<int> at_j;
  std::vector<const RRBuffers*> bufs;
  std::vector<int> jc;
  // one round's cycles of the problems in cyc, on stream st (stream-ordered after every
  // problem's set-up launches)
  std::vector<int> cyc_g[kMaxGroups];
  auto run_round = [&](const std::vector<int>& cyc, hipStream_t st) -> int {
    size_t L = 0;
    for (int i : cyc) L = std::max(L, sm[i].sv.plan.size());
    int r;
    for (size_t j = 0; j < L; ++j) {  // sweeps: the j-th of every plan
      at_j.clear();
      for (int i : cyc)
        if (j < sm[i].sv.plan.size()) at_j.push_back(i);
      r = groups(
          at_j,
          [&](int i) {
            const Solver& s = sm[i].sv;
            const Solver::PlanItem& x = s.plan[j];
            return std::make_tuple(s.pb, x.smode, x.has_step, x.q_ready, x.step.next_mode,
                                   s.w.sweep_ws != nullptr);
          },
          [&](const std::vector<int>& g, ProbBatch& b) {
            const Solver& A = sm[g[0]].sv;
            const Solver::PlanItem& x = A.plan[j];
            if (b.n == 1 || !A.w.sweep_ws)
              return apply_op(A.op, A.w, A.d, A.pb, st, x.smode, x.has_step ? &x.step : nullptr, x.q_ready);
            SweepBatch sb{};
            sb.n = b.n;
            for (int m = 0; m < b.n; ++m) {
              const SweepStep& y = sm[g[m]].sv.plan[j].step;
              sb.off[m] = b.off[m];
              sb.kind[m] = y.kind;
              sb.tau[m] = y.tau;
              sb.thr[m] = y.thr;
              sb.a[m] = y.a;
              sb.cc[m] = y.cc;
              sb.gamma[m] = y.gamma;
            }
            const int64_t ld = 2 * A.pb;
            return sweep_apply(A.w.rr.Z, A.d, A.pb, ld, A.w.rr.Z + A.pb, ld, 1.f, A.w.sweep_ws,
                               A.w.sweep_bytes, st, x.smode, x.has_step ? &x.step : nullptr, x.q_ready,
                               false, &sb);
          });
      if (r) return r;
    }
    // Grams
    r = groups(cyc, [&](int i) { return sm[i].sv.pb; },
               [&](const std::vector<int>& g, ProbBatch& b) {
                 const Solver& A = sm[g[0]].sv;
                 const int n2 = 2 * A.pb;
                 return skinny_launch(true, A.w.rr.Z, n2, A.w.rr.Z, n2, A.w.rr.C, n2, n2, n2, A.d, 1.f,
                                      0.f, A.w.slab, A.w.slab_bytes, st, &b);
               });
    if (r) return r;
    // small solves: one launch per subspace width (the last block of k > 128 pairs may
    // be narrower)
    for (size_t a = 0; a < cyc.size(); ++a) {
      const int pw = sm[cyc[a]].sv.pb;
      bool seen = false;
      for (size_t c = 0; c < a; ++c) seen |= sm[cyc[c]].sv.pb == pw;
      if (seen) continue;
      bufs.clear();
      jc.clear();
      for (int i : cyc)
        if (sm[i].sv.pb == pw) {
          bufs.push_back(&sm[i].sv.w.rr);
          jc.push_back(sm[i].sv.jcap);
        }
      if ((r = rr_small_batch_launch(bufs.data(), jc.data(), (int)bufs.size(), pw, st))) return r;
    }
    // Ritz vectors, residuals and the status blocks
    return groups(
        cyc, [&](int i) { return std::make_tuple(sm[i].sv.pb, sm[i].sv.kc, sm[i].sv.ldv); },
        [&](const std::vector<int>& g, ProbBatch& b) {
          const Solver& A = sm[g[0]].sv;
          for (int m = 0; m < b.n; ++m) {
            b.V[m] = sm[g[m]].sv.Vb;
            b.evals[m] = sm[g[m]].sv.evb;
            b.hs[m] = sm[g[m]].sv.hs;
          }
          int r2 = rr_update_batch_launch(A.w.rr, A.d, A.pb, A.kc, A.ldv, b, st);
          if (r2) return r2;
          hipLaunchKernelGGL(status_kernel, dim3((unsigned)b.n), dim3(256), 0, st, A.w.rr.resid, A.kc + 1,
                             A.w.rr.lam, A.pb, A.w.rr.info, b);
          DEIG_HIP_CHECK(hipGetLastError());
          return (int)DEIG_OK;
        });
  };
  // group g's problems to their next cycle (or DONE), then its round enqueued
  auto advance = [&](int g) -> int {
    std::vector<int>& cy = cyc_g[g];
    cy.clear();
    int r = DEIG_OK;
    for (int i = g; i < W && !r; i += NG) {
      SolveSM& m = sm[i];
      while (m.state != SolveSM::DONE) {
        if ((r = m.settle()) || m.state == SolveSM::DONE) break;
        bool ended = false;
        m.sv.plan_cycle(&ended);
        if (!ended) {
          cy.push_back(i);
          break;
        }
        if ((r = m.end_block())) break;
      }
      if (r) m.rc = r;
    }
    if (r || cy.empty()) return r;
    return run_round(cy, gs[g]);
  };
  for (int g = 0; g < NG && !rc; ++g) rc = advance(g);
  auto pending = [&]() {
    for (int g = 0; g < NG; ++g)
      if (!cyc_g[g].empty()) return true;
    return false;
  };
  while (!rc && pending()) {
    for (int g = 0; g < NG && !rc; ++g) {
      if (cyc_g[g].empty()) continue;
      if (hipStreamSynchronize(gs[g]) != hipSuccess) {
        rc = fail(DEIG_EHIP, "solve_batch: stream synchronisation failed");
        break;
      }
      for (int i : cyc_g[g]) {
        bool done = false;
        if (!(rc = sm[i].sv.cycle_finish(&done)) && done) rc = sm[i].end_block();
        if (rc) {
          sm[i].rc = rc;
          break;
        }
      }
      if (!rc) rc = advance(g);
    }
  }
  {
    const int rj = join();
    if (rj && !rc) rc = rj;
  }
  if (rc) {
    char msg[1024];
    snprintf(msg, sizeof(msg), "%s", g_err);
    for (int i = 0; i < W; ++i) {
      if (sweeps_out) sweeps_out[i] = sm[i].sv.it;
      if (resid_out) resid_out[i] = sm[i].sv.last;
      if (status_out) status_out[i] = sm[i].rc ? sm[i].rc : rc;
    }
    set_error("%s", msg);
    return rc;
  }
  int first = DEIG_OK;
  char msg[1024] = "";
  for (int i = 0; i < W; ++i) {
    const int r = sm[i].outcome(sweeps_out ? sweeps_out + i : nullptr, resid_out ? resid_out + i : nullptr);
    if (status_out) status_out[i] = r;  // each problem's own outcome, as solve() would return it
    if (r && !first) {
      first = r;
      snprintf(msg, sizeof(msg), "%s", g_err);
    }
  }
  if (first) set_error("%s", msg);
  return first;
}

}  // namespace
}  // namespace deig

using namespace deig;

extern "C" {

int deig_version(void) { return 0x000600; }

void deig_shutdown(void) {
  // nothing allocated (no solver ran in this process): make no HIP call at all
  if (status_pool().empty()) return;
  (void)hipDeviceSynchronize();
  status_pool().drain();
  (void)hipGetLastError();
}

const char* deig_last_error(void) { return g_err; }

void deig_solver_opts_init(deig_solver_opts* o) {
  if (!o) return;
  memset(o, 0, sizeof(*o));
  o->size = (int)sizeof(deig_solver_opts);
  o->sweep_algo = DEIG_SWEEP_AUTO;
  o->rr_every = 0;
  o->chebyshev = 1;
  o->cheb_above = -1.f;
  o->deflate = 1;
  o->deflate_early = 1;
  o->jacobi_early_sweeps = -1;
  o->jacobi_early_above = -1.f;
  o->fast_until = 1e-3f;
  o->round_until = 1e-4f;
  o->debug = 0;
  o->half_until = 1e-2f;
}

// An explicit S the solver reads in place needs lds % 4 == 0 and 16-byte alignment;
// a staged one (solver_dims: d % 4 != 0, d < 16, subspace wider than d) only its
// element alignment.
static int check_matrix(const void* S, int stype, int64_t d, int k, int p, int64_t lds,
                        const char* what) {
  if (!S || lds < d) return fail(DEIG_EINVAL, "%s: need S with lds >= d", what);
  if (k < 1 || k > d) return fail(DEIG_EINVAL, "%s: need 1 <= k <= d (k=%d, d=%lld)", what, k, (long long)d);
  const Dims dm = solver_dims(d, k, p, false);
  const uintptr_t a = reinterpret_cast<uintptr_t>(S);
  if (dm.staged) {
    if (a % (stype == DEIG_F64 ? 8 : 4))
      return fail(DEIG_EINVAL, "%s: S must be aligned to its element size", what);
  } else if (lds % 4 != 0 || !aligned16(S)) {
    return fail(DEIG_EINVAL, "%s: S must be 16-byte aligned with lds %% 4 == 0", what);
  }
  return DEIG_OK;
}

static int check_opts(const deig_solver_opts* o) {
  if (o && o->size != (int)sizeof(deig_solver_opts))
    return fail(DEIG_EINVAL, "solver options: size %d != %d (call deig_solver_opts_init)", o->size,
                (int)sizeof(deig_solver_opts));
  return DEIG_OK;
}

static int syrk_resolve(int64_t n, int algo) {
  if (algo != DEIG_SYRK_AUTO) return algo;
  return n >= DEIG_SYRK_SPLIT_MIN_ROWS ? DEIG_SYRK_SPLIT3 : DEIG_SYRK_FP32;
}

size_t deig_syrk_workspace_ex(int64_t n, int64_t d, int algo) {
  algo = syrk_resolve(n, algo & ~DEIG_SYRK_ACCUMULATE);
  if (algo == DEIG_SYRK_FP32) return syrk_workspace_bytes(n, d);
  if (algo == DEIG_SYRK_SPLIT3) return syrk_split_workspace_bytes(n, d);
  return 0;
}

int deig_syrk_f32_ex(const float* X, int64_t n, int64_t d, int64_t ldx, float alpha, float* S,
                     int64_t lds, int algo, void* ws, size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  const bool acc = (algo & DEIG_SYRK_ACCUMULATE) != 0;
  algo = syrk_resolve(n, algo & ~DEIG_SYRK_ACCUMULATE);
  if (acc && algo != DEIG_SYRK_SPLIT3)
    return fail(DEIG_EINVAL, "syrk: DEIG_SYRK_ACCUMULATE needs the split3 algorithm");
  if (algo == DEIG_SYRK_FP32)
    return syrk_launch(X, n, d, ldx, alpha, S, lds, ws, ws_bytes, (hipStream_t)stream);
  if (algo == DEIG_SYRK_SPLIT3)
    return syrk_split_launch(X, n, d, ldx, alpha, S, lds, ws, ws_bytes, (hipStream_t)stream, acc);
  return fail(DEIG_EINVAL, "syrk: unknown algorithm %d", algo);
}

size_t deig_syrk_workspace(int64_t n, int64_t d) {
  return deig_syrk_workspace_ex(n, d, DEIG_SYRK_DEFAULT);
}

int deig_syrk_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float alpha, float* S,
                  int64_t lds, void* ws, size_t ws_bytes, void* stream) {
  return deig_syrk_f32_ex(X, n, d, ldx, alpha, S, lds, DEIG_SYRK_DEFAULT, ws, ws_bytes, stream);
}

size_t deig_syrk_shift_workspace(int64_t n, int64_t d, int xtype) {
  return syrk_shift_workspace_bytes(n, d, xtype);
}

int deig_syrk_shift(const void* X, int xtype, int64_t n, int64_t d, int64_t ldx, double alpha,
                    double* S64, int64_t lds64, float* S, int64_t lds, void* ws, size_t ws_bytes,
                    void* stream) {
  g_err[0] = 0;
  return syrk_shift_launch(X, xtype, n, d, ldx, alpha, S64, lds64, S, lds, ws, ws_bytes,
                           (hipStream_t)stream);
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

int deig_default_subspace(int64_t d, int k) { return default_subspace(d, k); }

static size_t topk_ws(int64_t d, int k, int p, bool implicit, int64_t mk, const deig_solver_opts* o,
                      int stype = DEIG_F32) {
  const Opts oo = make_opts(o);
  if (d < 1 || k < 1) return 0;
  const Dims dm = solver_dims(d, k, p, implicit);
  int pb = dm.pb, kb = dm.kb;
  if (pb < 16) pb = 16;
  if (kb < 1) kb = 1;
  const bool image = !implicit && oo.sweep_algo != DEIG_SWEEP_FP32;
  Carve c(nullptr, 0);
  carve_stage(c, dm, k, stype);
  size_t total = 0;
  carve_solver(nullptr, 0, dm.dp, kb, k, pb, implicit ? mk : 0, image, &total);
  return c.off + total;
}

size_t deig_topk_workspace_ex(int64_t d, int k, int p, int stype, const deig_solver_opts* opts) {
  return topk_ws(d, k, p, false, 0, opts, stype);
}

size_t deig_topk_workspace(int64_t d, int k, int p) { return topk_ws(d, k, p, false, 0, nullptr); }

int deig_topk_sym_ex(const void* S, int stype, int64_t d, int64_t lds, int k, int p, int max_sweeps,
                     float tol, const float* Q0, int k0, int64_t ldq0, float* V, int64_t ldv,
                     float* evals, int* sweeps_out, float* resid_out, const deig_solver_opts* opts,
                     void* ws, size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  if (int rc = check_opts(opts)) return rc;
  if (stype != DEIG_F32 && stype != DEIG_F64)
    return fail(DEIG_EINVAL, "topk: unknown element type %d", stype);
  if (int rc = check_matrix(S, stype, d, k, p, lds, "topk")) return rc;
  Operator op{};
  op.implicit = false;
  op.S = S;
  op.stype = stype;
  op.lds = lds;
  return solve(op, d, k, p, max_sweeps, tol, Q0, k0, ldq0, V, ldv, evals, sweeps_out, resid_out,
               make_opts(opts), ws, ws_bytes, (hipStream_t)stream);
}

int deig_topk_sym_f32(const float* S, int64_t d, int64_t lds, int k, int p, int max_sweeps,
                      float tol, const float* Q0, int k0, int64_t ldq0, float* V, int64_t ldv,
                      float* evals, int* sweeps_out, float* resid_out, void* ws, size_t ws_bytes,
                      void* stream) {
  return deig_topk_sym_ex(S, DEIG_F32, d, lds, k, p, max_sweeps, tol, Q0, k0, ldq0, V, ldv, evals,
                          sweeps_out, resid_out, nullptr, ws, ws_bytes, stream);
}

size_t deig_topk_batch_workspace(int W, int64_t d, int k, int p, int stype,
                                 const deig_solver_opts* opts) {
  if (W < 1) return 0;
  return (size_t)W * align_up(topk_ws(d, k, p, false, 0, opts, stype), 256);
}

int deig_topk_sym_batch(int W, const void* const* S, int stype, int64_t d, int64_t lds, int k, int p,
                        int max_sweeps, float tol, float* const* V, int64_t ldv, float* const* evals,
                        int* sweeps_out, float* resid_out, const deig_solver_opts* opts, void* ws,
                        size_t ws_bytes, void* const* streams, void* stream) {
  (void)streams;  // r03's per-problem streams: every launch is on `stream` since r04
  return deig_topk_sym_batch_ex(W, S, stype, d, lds, k, p, max_sweeps, tol, V, ldv, evals, sweeps_out,
                                resid_out, nullptr, opts, ws, ws_bytes, stream);
}

int deig_topk_sym_batch_ex(int W, const void* const* S, int stype, int64_t d, int64_t lds, int k, int p,
                           int max_sweeps, float tol, float* const* V, int64_t ldv,
                           float* const* evals, int* sweeps_out, float* resid_out, int* status_out,
                           const deig_solver_opts* opts, void* ws, size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  if (int rc = check_opts(opts)) return rc;
  if (W < 1 || !S || !V || !evals) return fail(DEIG_EINVAL, "topk_batch: need W >= 1 and S / V / evals arrays");
  if (stype != DEIG_F32 && stype != DEIG_F64)
    return fail(DEIG_EINVAL, "topk_batch: unknown element type %d", stype);
  for (int i = 0; i < W; ++i)
    if (int rc = check_matrix(S[i], stype, d, k, p, lds, "topk_batch")) return rc;
  const size_t each = align_up(topk_ws(d, k, p, false, 0, opts, stype), 256);
  if (!ws || ws_bytes < (size_t)W * each)
    return fail(DEIG_EWORKSPACE, "topk_batch: workspace %zu bytes < required %zu", ws_bytes,
                (size_t)W * each);
  std::vector<Operator> ops(W);
  for (int i = 0; i < W; ++i) {
    ops[i] = Operator{};
    ops[i].implicit = false;
    ops[i].S = S[i];
    ops[i].stype = stype;
    ops[i].lds = lds;
  }
  return solve_batch(W, ops.data(), d, k, p, max_sweeps, tol, V, ldv, evals, sweeps_out, resid_out,
                     status_out, make_opts(opts), static_cast<char*>(ws), each, (hipStream_t)stream);
}

size_t deig_projavg_workspace_ex(int64_t d, int64_t mk, int k, int p,
                                 const deig_solver_opts* opts) {
  return topk_ws(d, k, p, true, mk, opts);
}

size_t deig_projavg_workspace(int64_t d, int64_t mk, int k, int p) {
  return topk_ws(d, k, p, true, mk, nullptr);
}

int deig_projavg_topk_ex(const float* Wt, int64_t d, int64_t mk, int64_t ldw, float scale, int k,
                         int p, int max_sweeps, float tol, const float* Q0, int k0, int64_t ldq0,
                         float* V, int64_t ldv, float* evals, int* sweeps_out, float* resid_out,
                         const deig_solver_opts* opts, void* ws, size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  if (int rc = check_opts(opts)) return rc;
  if (!Wt || mk < 1 || ldw < d || ldw % 4 != 0 || !aligned16(Wt))
    return fail(DEIG_EINVAL, "projavg: Wt must be 16-byte aligned, mk >= 1, ldw >= d, ldw %% 4 == 0");
  Operator op{};
  op.implicit = true;
  op.stype = DEIG_F32;
  op.Wt = Wt;
  op.mk = mk;
  op.ldw = ldw;
  op.scale = scale;
  return solve(op, d, k, p, max_sweeps, tol, Q0, k0, ldq0, V, ldv, evals, sweeps_out, resid_out,
               make_opts(opts), ws, ws_bytes, (hipStream_t)stream);
}

int deig_projavg_topk_f32(const float* Wt, int64_t d, int64_t mk, int64_t ldw, float scale, int k,
                          int p, int max_sweeps, float tol, const float* Q0, int k0, int64_t ldq0,
                          float* V, int64_t ldv, float* evals, int* sweeps_out, float* resid_out,
                          void* ws, size_t ws_bytes, void* stream) {
  return deig_projavg_topk_ex(Wt, d, mk, ldw, scale, k, p, max_sweeps, tol, Q0, k0, ldq0, V, ldv,
                              evals, sweeps_out, resid_out, nullptr, ws, ws_bytes, stream);
}

int deig_sym_power_f32(const float* S, int64_t d, int64_t lds, float* Q, int p, int64_t ldq,
                       float* Y, int64_t ldy, const float* cs, int steps, int algo, void* ws,
                       size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  DEIG_REQUIRE(steps >= 1 && cs && Q, "sym_power: need steps >= 1, cs and Q");
  const bool prepared = (algo & DEIG_SWEEP_PREPARED) != 0;
  const int smode = (algo & DEIG_SWEEP_HALF)      ? kSweepHalf
                    : (algo & DEIG_SWEEP_FAST)    ? kSweepFast
                    : (algo & DEIG_SWEEP_ROUND_Q) ? kSweepRoundQ
                                                  : kSweepExact;
  algo &= ~(DEIG_SWEEP_PREPARED | DEIG_SWEEP_ROUND_Q | DEIG_SWEEP_FAST | DEIG_SWEEP_HALF);
  if (algo != DEIG_SWEEP_AUTO && algo != DEIG_SWEEP_BF16X6)
    return fail(DEIG_EINVAL, "sym_power: algorithm %d has no fused chain (bf16x6 only)", algo);
  hipStream_t st = (hipStream_t)stream;
  if (!prepared) {
    const int rc = sweep_prepare(S, DEIG_F32, d, lds, p, ws, ws_bytes, st);
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
    step.write_y = i + 1 == steps;  // the contract: on return Y = S Q_{steps-1}
    const int rc = sweep_apply(Q, d, p, ldq, Y, ldy, 1.f, ws, ws_bytes, st, smode, &step, i > 0);
    if (rc) return rc;
  }
  return DEIG_OK;
}

size_t deig_sym_apply_workspace(int64_t d, int p, int algo) {
  algo &= ~(DEIG_SWEEP_PREPARED | DEIG_SWEEP_ROUND_Q | DEIG_SWEEP_FAST | DEIG_SWEEP_HALF |
            DEIG_SWEEP_KERNEL_ONLY);
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
  const int smode = (algo & DEIG_SWEEP_HALF)      ? kSweepHalf
                    : (algo & DEIG_SWEEP_FAST)    ? kSweepFast
                    : (algo & DEIG_SWEEP_ROUND_Q) ? kSweepRoundQ
                                                  : kSweepExact;
  algo &= ~(DEIG_SWEEP_PREPARED | DEIG_SWEEP_ROUND_Q | DEIG_SWEEP_FAST | DEIG_SWEEP_HALF |
            DEIG_SWEEP_KERNEL_ONLY);
  if (algo != DEIG_SWEEP_AUTO && algo != DEIG_SWEEP_BF16X6)
    return fail(DEIG_EINVAL, "sym_apply: unknown algorithm %d", algo);
  if (!prepared) {
    const int rc = sweep_prepare(S, DEIG_F32, d, lds, p, ws, ws_bytes, (hipStream_t)stream);
    if (rc) return rc;
  }
  return sweep_apply(Q, d, p, ldq, Y, ldy, alpha, ws, ws_bytes, (hipStream_t)stream, smode,
                     nullptr, kernel_only, kernel_only);
}

size_t deig_oja_workspace(int64_t b, int64_t d, int k) { return oja_workspace_bytes(b, d, k); }

int deig_oja_steps_ex(const float* X, int64_t nb, int64_t b, int64_t d, int64_t ldx, float eta,
                      float* V, int k, int64_t ldv, int orth_every, int algo, void* ws,
                      size_t ws_bytes, void* stream) {
  g_err[0] = 0;
  if (!X || !V || !aligned16(X)) return fail(DEIG_EINVAL, "oja: X must be 16-byte aligned");
  return oja_steps_launch(X, nb, b, d, ldx, eta, V, k, ldv, orth_every, ws, ws_bytes,
                          (hipStream_t)stream, algo);
}

int deig_oja_error(const void* ws, size_t ws_bytes, int64_t b, int64_t d, int k, void* stream) {
  g_err[0] = 0;
  return oja_error(ws, ws_bytes, b, d, k, (hipStream_t)stream);
}

int deig_oja_steps_f32(const float* X, int64_t nb, int64_t b, int64_t d, int64_t ldx, float eta,
                       float* V, int k, int64_t ldv, int orth_every, void* ws, size_t ws_bytes,
                       void* stream) {
  return deig_oja_steps_ex(X, nb, b, d, ldx, eta, V, k, ldv, orth_every, DEIG_OJA_AUTO, ws,
                           ws_bytes, stream);
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
