# decode-step kernel census after the layer ops (what the remaining 3.2 ms/token is made of)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_decode2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_decode2 -- python3 bench.py --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline > gpurun_out/prof_decode2.log 2>&1 || exit $?
tail -1 gpurun_out/prof_decode2.log | cut -c1-300
