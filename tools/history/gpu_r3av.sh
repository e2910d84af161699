# reference algorithm (HF GPT2LMHeadModel, default SDPA attention now that the native init no longer flips the shared config to eager) vs native, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3av
timeout -k 10 400 python bench.py --impl reference --steps 3 --warmup 1 2> gpurun_out/r3av/ref.err | tail -1 > gpurun_out/r3av/ref.json || { tail -20 gpurun_out/r3av/ref.err; exit 1; }
timeout -k 10 300 python bench.py --steps 8 --warmup 2 2> gpurun_out/r3av/nat.err | tail -1 > gpurun_out/r3av/nat.json || { tail -20 gpurun_out/r3av/nat.err; exit 1; }
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3av/prof -o prof -- python3 bench.py --impl reference --steps 1 --warmup 1 > gpurun_out/r3av/prof.log 2>&1 || exit 1
for f in ref nat; do python -c "import json;d=json.load(open('gpurun_out/r3av/$f.json'));print('$f',d['value'],d['ms_per_step'],d.get('phase_ms_per_step'))"; done
