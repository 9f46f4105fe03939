# is the force-shard graph-capture failure caused by the layer ops? (TP path at world size 1)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511"
timeout -k 10 300 $TR bench.py --force-shard --no-prefill --no-cpu --no-roofline --no-layer-ops > gpurun_out/fs_nolo.log 2>&1
echo "no-layer-ops rc=$?"; grep -E '^\{|graph decode failed' gpurun_out/fs_nolo.log | cut -c1-200
