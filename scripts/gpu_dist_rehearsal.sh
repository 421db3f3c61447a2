set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_BACKEND=gloo BENCH_BATCH=8 timeout -k 10 600 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/dist2.log 2>&1 || { echo "dist rehearsal failed"; tail -30 gpurun_out/dist2.log; exit 1; }
grep metric gpurun_out/dist2.log
timeout -k 10 600 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/dist1.log 2>&1 || { echo "torchrun n1 failed"; tail -30 gpurun_out/dist1.log; exit 1; }
grep metric gpurun_out/dist1.log
