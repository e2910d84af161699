cd $GRAFT_REPO_ROOT
for a in "--rocm_fa ck" "--rocm_fa aotriton" "--dropout 0.0" "--dropout 0.0 --rocm_fa ck"; do
  echo "== $a"; timeout -k 10 300 python bench.py --steps 3 --warmup 1 $a 2>&1 | grep -E '^\{|Error|error' | cut -c1-200
done
