# Round-4 GPU pass i: stagger between the two co-resident workgroups of the 128-row rows tile.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_i
mkdir -p $O
timeout -k 10 400 python scripts/ab_mlp_inproc.py --stagger 0,1,2,3,5 --rounds 6 --steps 50 > $O/ab_stagger.json 2>&1 || exit 1
python - <<'PY'
import json
t=open('gpurun_out/r04_i/ab_stagger.json').read(); d=json.loads(t[t.index('{'):])
print({k: round(v['median_us'], 2) for k, v in d.items() if 'median_us' in v})
PY
echo r04_i done
