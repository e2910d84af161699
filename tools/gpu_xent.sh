set -o pipefail
cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-reg p512 p1024}; do
  echo "== $v"; DLION_XENT=$v timeout -k 10 120 python tools/bench_xent.py || exit 1
  DLION_XENT=$v timeout -k 10 120 python tools/bench_xent.py 8192 32000 || exit 1
done
