set -o pipefail
cd $GRAFT_REPO_ROOT
for a in "--warmup 3 --steps 20" "--warmup 200 --steps 1000" "--warmup 3 --steps 20" "--warmup 2000 --steps 2000"; do
timeout -k 10 200 python bench.py --no-cpu-baseline $a 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['roofline']['kernel_ms'])" || exit 1
done
