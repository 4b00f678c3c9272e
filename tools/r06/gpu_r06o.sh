#!/bin/bash
# r06o: host UMEM registrations reference-counted across queues (several
# queues over one host buffer, as the latency harness's workers): the -m gpu suite once (new shared-UMEM test), then
# the drop-in latency sweep with 1 and 3 workers (r06n's 3-worker run failed
# at teardown: the second queue's hipHostUnregister found no registration).
set -e
tag=${1:-r06o}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
timeout -k 10 600 python3 -u tools/dropin_latency.py --out gpurun_out/dropin_$tag.jsonl > gpurun_out/dropin_$tag.log 2>&1
