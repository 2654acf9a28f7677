#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/det
mkdir -p $O
cd $R
timeout -k 10 200 python -u scripts/det_check.py $O/new1.json 30 > $O/n1.log 2>&1 &&
timeout -k 10 200 python -u scripts/det_check.py $O/new2.json 30 > $O/n2.log 2>&1 &&
PYTHONPATH=$R/_ab_old timeout -k 10 200 python -u scripts/det_check.py $O/old1.json 30 > $O/o1.log 2>&1 &&
PYTHONPATH=$R/_ab_old timeout -k 10 200 python -u scripts/det_check.py $O/old2.json 30 > $O/o2.log 2>&1
rc=$?
python - <<'PY'
import json
d = {k: json.load(open(f"gpurun_out/det/{k}.json")) for k in ("new1", "new2", "old1", "old2")}
for k, v in d.items(): print(k, v[-1])
def same(a, b, key): return all(x[key] == y[key] for x, y in zip(d[a][:-1], d[b][:-1]))
for a, b in (("new1", "new2"), ("old1", "old2"), ("new1", "old1")):
    print(a, b, {key: same(a, b, key) for key in ("hip_loss", "hip_prio", "t32_loss")})
PY
exit $rc
