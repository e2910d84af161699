# r6 call 7: LM-head input gradient through the timed pick (own NT vs searched hipBLASLt) -- bench A/B,
# "own" = the pick pre-seeded with the own NT kernel (the previous fixed choice)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c7; mkdir -p $O
ab() {
  timeout -k 10 300 python3 -c "
import sys, runpy
from distributed_lion_pytorch_amd.ops import linear
if '$1' == 'own':
    linear._GEMM_PICK[('fwd', 20480, 768, 50304, 50304, 50304, False)] = 'own'
sys.argv = ['bench.py', '--steps', '20', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
print('pick', {k: v for k, v in linear._GEMM_PICK.items() if k[0] == 'fwd' and k[3] == 50304}, file=sys.stderr)
" 2> $O/err_$1_$2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ms_per_step'])"
}
for r in 1 2 3; do ab own $r || exit 1; ab pick $r || exit 1; done | tee $O/bench_ab.txt
grep pick $O/err_pick_1.log
