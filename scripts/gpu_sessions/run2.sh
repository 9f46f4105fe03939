set -u
cd $GRAFT_REPO_ROOT
SKIP_SMOKE=1 SKIP_BENCH=1 bash scripts/gpu_check.sh || exit $?
DECODE_CMD="python3 bench.py --steps 8 --warmup 2 --no-cpu --no-roofline" bash scripts/gpu_profile.sh
