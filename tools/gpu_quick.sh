set -e
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pinned.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or pinned or stage or full_size" > gpurun_out/pytest_gpu_s5.log 2>&1
timeout -k 10 300 python3 bench.py --no-9000 --cpu-baseline-sec 2 > gpurun_out/bench_s5.json 2> gpurun_out/bench_s5.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-9000 > gpurun_out/prof_s5.log 2>&1
