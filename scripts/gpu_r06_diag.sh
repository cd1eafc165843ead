# Round 6 diagnosis of k_run's memory stalls on the tlv headline: the
# gfx950 counter list, then PMC passes (one block's limits per pass) for the
# vector L1 / UTCL1 (GPU address translation) and L2 hit rates.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && mkdir -p $R/gpurun_out/diag
timeout -s KILL 120 rocprofv3 -L > $R/gpurun_out/diag/counters.txt 2>&1 || { echo LIST_FAIL; tail -5 $R/gpurun_out/diag/counters.txt; exit 1; }
grep -o "TCP_UTCL[A-Z0-9_]*\|TCC_HIT[A-Za-z0-9_]*\|TCC_MISS[A-Za-z0-9_]*\|TCP_[A-Z_]*STALL[A-Z_]*\|TA_BUSY[a-z_]*\|UTCL2[A-Z0-9_]*" $R/gpurun_out/diag/counters.txt | sort -u > $R/gpurun_out/diag/names.txt
cat $R/gpurun_out/diag/names.txt | tr '\n' ' '; echo
pass() {  # name counters...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d /tmp/diag/$n -o run -- python3 $R/scripts/prof_leg.py tlv ${STEPS:-8} > $R/gpurun_out/diag/$n.log 2>&1 || { echo "PASS_FAIL $n"; tail -5 $R/gpurun_out/diag/$n.log; exit 1; }
  f=$(find /tmp/diag/$n -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_run' in r.get('Kernel_Name', '')]
tot = collections.defaultdict(float); disp = collections.defaultdict(set)
for r in rows:
    tot[r['Counter_Name']] += float(r['Counter_Value']); disp[r['Counter_Name']].add(r['Dispatch_Id'])
print(sys.argv[2], {k: (round(v / max(1, len(disp[k]))), len(disp[k])) for k, v in tot.items()})
PY
  rm -rf /tmp/diag/$n
}
for p in "$@"; do pass ${p%%=*} $(echo ${p#*=} | tr "," " "); done
