# rocprofv3 kernel-trace + stats of a short 1-GPU bench run.  Usage: bash tools/profile_bench.sh <tag> [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o prof -- python3 bench.py --steps 2 --warmup 1 "$@" > gpurun_out/prof_$TAG/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_$TAG/bench.log
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -30 {}'
