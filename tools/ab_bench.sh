# Same-box A/B of bench.py: bash tools/ab_bench.sh "<env A>" "<env B>" [rounds] [bench args]
# e.g. bash tools/ab_bench.sh "DLION_DGELU_GEMM=0 DLION_GELU_GEMM=0" "" 2 --steps 8
set -o pipefail
cd $GRAFT_REPO_ROOT
A=$1; B=$2; R=${3:-2}; shift 3
for i in $(seq $R); do
  for tag in A B; do
    envs=$([ $tag = A ] && echo "$A" || echo "$B")
    v=$(env $envs timeout -k 10 300 python bench.py "$@" 2>/dev/null | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])") || exit 1
    echo "$tag [$envs] $v"
  done
done
