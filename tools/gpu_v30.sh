set -e
mkdir -p gpurun_out/ab_v30
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_v30.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_v30/k4_$r.json 2> gpurun_out/ab_v30/k4_$r.err
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --histo-eager > gpurun_out/ab_v30/eager_$r.json 2> gpurun_out/ab_v30/eager_$r.err
done
timeout -k 10 200 python3 bench.py --frame-len 9000 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_v30/k1_9000.json 2> gpurun_out/ab_v30/k1_9000.err
