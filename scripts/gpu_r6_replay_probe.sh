# round 6: host submission cost of one decode graph replay (benchmarks/probe_replay_host.py) under the HIP runtime's
# graph-launch settings, and with one vs two batch-slice chains
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # $1: tag, rest: env assignments
  tag=$1; shift
  env "$@" timeout -k 10 240 python3 benchmarks/probe_replay_host.py > gpurun_out/probe_$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/probe_$tag.log; return 1; }
  echo "$tag $(grep '^{' gpurun_out/probe_$tag.log)"
}
case "${1:-all}" in
all)
run default && \
run capture0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && \
run capture1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && \
run queues1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && \
run parts1 PROBE_PARTS=1 && \
run parts1_capture1 PROBE_PARTS=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && \
run batch64 DEBUG_HIP_GRAPH_BATCH_SIZE=64 ;;
perpart)
run default && run perpart PROBE_PERPART=1 && run parts1 PROBE_PARTS=1 && run perpart_b PROBE_PERPART=1 ;;
esac
