# r6 call 21: steady-state check -- a 300-step GPT-2 bench (same process, no drift / leak in ms per
# step or peak memory) next to the 20-step driver form, and a 40-step Llama-3-8B run
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c21; mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/b20.json 2> $O/b20.err || { tail -5 $O/b20.err; exit 1; }
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 > $O/b300.json 2> $O/b300.err || { tail -5 $O/b300.err; exit 1; }
timeout -k 10 400 python3 bench.py --task llama3 --steps 40 --warmup 3 > $O/llama40.json 2> $O/llama40.err || { tail -5 $O/llama40.err; exit 1; }
for f in b20 b300 llama40; do tail -1 $O/$f.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d.get('peak_memory_gb', d.get('max_memory_allocated_gb')))"; done
