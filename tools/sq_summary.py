"""SQ counter summary of the conv kernels from rocprofv3 --pmc passes
(tools/gpu_r04a.sh: sq1 = wave-cycle split + MFMA busy, sq2 = instruction
counts + LDS, sq3 = active-instruction cycles).

    python tools/sq_summary.py gpurun_out/r04a > profiles/r04a_sq_conv_summary.md

Per kernel (averaged over its dispatches): the fractions of wave cycles a
wave spends parked on s_waitcnt / s_barrier (SQ_WAIT_ANY), stalled at issue
(SQ_WAIT_INST_ANY: the MFMA pipe busy or a dependency), issuing
(SQ_ACTIVE_INST_ANY); MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES over
GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs, as tools/pmc_summary.py); VALU (incl.
MFMA), LDS and SALU instructions per MFMA; LDS bank-conflict cycles over
LDS-active cycles."""
import collections
import csv
import os
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in ('sq1', 'sq2', 'sq3'):
        p = os.path.join(d, sub, 'p_counter_collection.csv')
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '') + ' grid ' + r['Grid_Size']
            agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
    return agg


def main():
    d = sys.argv[1]
    agg = load(d)
    print('| kernel | WAIT_ANY | WAIT_INST_ANY | ACTIVE_INST_ANY | MFMA util | VALU/MFMA | LDS/MFMA | SALU/MFMA '
          '| LDS conflict / active |')
    print('|---|---|---|---|---|---|---|---|---|')
    for k, v in sorted(agg.items()):
        if not v.get('SQ_INSTS_MFMA') or not any(v['SQ_INSTS_MFMA']):
            continue
        m = lambda c: sum(v[c]) / len(v[c]) if v.get(c) else float('nan')   # noqa: E731
        wc = m('SQ_WAVE_CYCLES')
        util = m('SQ_VALU_MFMA_BUSY_CYCLES') / (m('GRBM_GUI_ACTIVE') / 8 * 1024)
        mf = m('SQ_INSTS_MFMA')
        print('| %s | %.3f | %.3f | %.3f | %.3f | %.2f | %.2f | %.2f | %.3f |' % (
            k, m('SQ_WAIT_ANY') / wc, m('SQ_WAIT_INST_ANY') / wc, m('SQ_ACTIVE_INST_ANY') / wc, util,
            m('SQ_INSTS_VALU') / mf, m('SQ_INSTS_LDS') / mf, m('SQ_INSTS_SALU') / mf,
            m('SQ_LDS_BANK_CONFLICT') / m('SQ_LDS_IDX_ACTIVE')))


if __name__ == '__main__':
    main()
