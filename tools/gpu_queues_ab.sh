# c1 (8 concurrent worker solves on 8 HIP streams) with 4 (default) and 8
# hardware queues per process.
mkdir -p gpurun_out/hwq
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench.py --config c1 --steps 10 --warmup 3 --no-cpu-baseline --no-alt > gpurun_out/hwq/c1_q$q.json 2> gpurun_out/hwq/c1_q$q.err || exit 1
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/hwq/c5_q8.json 2> gpurun_out/hwq/c5_q8.err || exit 1
