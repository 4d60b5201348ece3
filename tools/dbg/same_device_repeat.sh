#!/bin/bash
# Repeat the --same-device bench (2 ranks on GPU 0) and keep every run's pivot
# sequence, to compare against the config-3 fixture (diagnostic).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-samerep}; mkdir -p $O
for i in $(seq 1 ${N:-4}); do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
    --master-addr 127.0.0.1 --master-port $((29600 + i)) bench.py --gpus 2 --same-device \
    --steps ${STEPS:-4} --warmup ${WARM:-1} --cpu-seconds 0 --dump-history $O/hist$i.npy \
    > $O/run$i.log 2>&1
  rc=$?; echo "[run $i] rc=$rc"; tail -1 $O/run$i.log | cut -c1-120
  [ $rc != 0 ] && exit $rc
done
exit 0
