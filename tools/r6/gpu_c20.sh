# r6 call 20: TN window split sweep again after the K-loop address diet (is the model's pick still the fastest?)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c20; mkdir -p $O
timeout -k 10 400 python3 -u tools/bench_tn_splits.py > $O/tn_splits.txt 2>&1 || { tail -20 $O/tn_splits.txt; exit 1; }
grep -v amdgpu.ids $O/tn_splits.txt
