#!/bin/bash
# r04a: the new parity tests first (chunked / accumulate SYRK, integration stub,
# staged solver dims, batch status), then the whole GPU suite (no -x: every failure
# listed), smoke, the 2-rank gloo rehearsal line and c4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_syrk_chunks.py tests/test_gpu_integration_stub.py \
  "tests/test_gpu_general_solver.py::test_indefinite_padded_dimension" \
  "tests/test_gpu_general_solver.py::test_batch_status_is_per_problem" \
  "tests/test_gpu_general_solver.py::test_k_above_128_rank_deficient" \
  "tests/test_gpu_solver_robust.py::test_gap_099_meets_bars" > $OUT/new_tests.log 2>&1
rc=$?
tail -30 $OUT/new_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  --durations=15 > $OUT/gputests.log 2>&1
rc=$?
tail -25 $OUT/gputests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
cat $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --config c2 --steps 3 --warmup 1 \
  > $OUT/bench_gloo2_c2.json 2> $OUT/bench_gloo2_c2.err || { tail -20 $OUT/bench_gloo2_c2.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail $OUT/bench_c4.err; exit 1; }
python - <<'PY'
import json
for f in ("bench_gloo2_c2", "bench_c4"):
    d = json.load(open(f"gpurun_out/r04a/{f}.json"))
    print(f, d["value"], d.get("process_group"), d.get("breakdown"))
PY
