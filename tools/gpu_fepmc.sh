#!/bin/bash
# SQ counters of the frontend kernel (two PMC passes over tools/fe_bench.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/fepmc
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o p -- python tools/fe_bench.py 32 3 > $OUT/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/b -o p -- python tools/fe_bench.py 32 3 > $OUT/b.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
for d in ('a', 'b'):
    for f in glob.glob('gpurun_out/fepmc/%s/**/*counter_collection.csv' % d, recursive=True):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if 'logmel512' in r.get('Kernel_Name', ''):
                acc[r['Counter_Name']].append(float(r['Counter_Value']))
        for k, v in sorted(acc.items()):
            print(d, k, 'per-dispatch mean %.4g' % (sum(v) / max(1, len(v))), 'n=%d' % len(v))
PY
