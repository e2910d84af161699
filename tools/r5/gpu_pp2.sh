# ping-pong v2 A/B (tests + per-kernel times + fwd+bwd wall), then SQ counters of v2 vs the 4-wave kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r5/gpu_attn_pp.sh 3 || exit 1
bash tools/r5/gpu_pmc_pp.sh || exit 1
