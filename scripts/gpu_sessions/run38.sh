# force-shard (TP code path at world size 1) graph capture vs the layer ops: which op, and does
# capture_error_mode=thread_local (the RCCL watchdog thread queries events during capture) fix it
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511"
for v in "--layer-ops norm" "--layer-ops rope" "--capture-mode thread_local" "--capture-mode relaxed"; do
  timeout -k 10 300 $TR bench.py --force-shard --layers 4 --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline $v > gpurun_out/fs_var.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep -E '^\{|graph decode failed' gpurun_out/fs_var.log | cut -c1-140
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
done
exit 0
