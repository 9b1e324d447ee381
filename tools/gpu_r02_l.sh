# round 2: roctx ranges under rocprofv3 --marker-trace (no PMC in this pass), kernel stats alongside
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/marker -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vector-free --size 1e8 > gpurun_out/marker.log 2>&1; rc=$?
echo "marker rc=$rc"
[ $rc -eq 0 ] || { tail -20 gpurun_out/marker.log; exit $rc; }
python3 - <<'PY'
import csv, glob, collections
f = sorted(glob.glob('gpurun_out/marker/**/run_marker_api_trace.csv', recursive=True))
print(f)
if f:
    rows = list(csv.DictReader(open(f[-1])))
    print(rows[0].keys() if rows else None)
    c = collections.Counter(r.get('Function') or r.get('Name') or '?' for r in rows)
    print(c.most_common(10))
    d = collections.defaultdict(list)
    for r in rows:
        nm = r.get('Function') or r.get('Name')
        try:
            d[nm].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
        except Exception:
            pass
    for k, v in d.items():
        print(k, len(v), 'mean ms', sum(v) / len(v))
PY
