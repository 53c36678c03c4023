set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVES -d gpurun_out/pmc/a -o a --output-format csv -- ./tools/ubench/group_miller 6918 1 > gpurun_out/pmc/a.log 2>&1 || { tail -5 gpurun_out/pmc/a.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc/b -o b --output-format csv -- ./tools/ubench/group_miller 6918 1 > gpurun_out/pmc/b.log 2>&1 || { tail -5 gpurun_out/pmc/b.log; exit 1; }
for f in $(find gpurun_out/pmc -name "*counter_collection.csv"); do python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
agg={}
for r in rows:
    if 'miller' not in r['Kernel_Name']: continue
    agg[r['Counter_Name']]=agg.get(r['Counter_Name'],0)+float(r['Counter_Value'])
for k,v in sorted(agg.items()): print(k, v)
PY
done
