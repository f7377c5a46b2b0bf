"""Summarise a profile_round.sh run into profiles/<tag>_*.{json,md}.

Per kernel: calls and average duration (rocprofv3 --kernel-trace --stats),
average FETCH_SIZE / WRITE_SIZE per launch from the two separate --pmc passes.
Units / gfx950 corrections per /opt/skills/guides/MI355X_MICROARCH.md §HBM:
FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports exactly half
the bytes of a wide (16 B/lane) coalesced read, so hbm_read = 2 * FETCH_SIZE
* 1024 (both raw and corrected values are kept); WRITE_SIZE is exact for
16-B stores.

usage: python tools/pmc_summary.py gpurun_out/prof/exact r02_exact
       python tools/pmc_summary.py merge r02 r02_exact r02_x3
"""
import csv
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return name.split('(')[0].strip()


def main(src, tag):
    stats = list(csv.DictReader(open(os.path.join(src, 'kt', 'kt_kernel_stats.csv'))))
    out = {}
    for r in stats:
        out[short(r['Name'])] = {'calls': int(r['Calls']), 'avg_ns': float(r['AverageNs']),
                                 'pct': float(r['Percentage'])}
    for ctr, sub in (('FETCH_SIZE', 'pmc_fetch'), ('WRITE_SIZE', 'pmc_write')):
        acc = defaultdict(list)
        p = os.path.join(src, sub, 'pmc_counter_collection.csv')
        for r in csv.DictReader(open(p)):
            if r['Counter_Name'] == ctr:
                acc[short(r['Kernel_Name'])].append(float(r['Counter_Value']))
        for k, v in acc.items():
            out.setdefault(k, {})[ctr.lower() + '_kib_avg'] = sum(v) / len(v)
    mp = os.path.join(src, 'pmc_mfma', 'pmc_counter_collection.csv')
    if os.path.exists(mp):
        acc = defaultdict(lambda: defaultdict(list))
        for r in csv.DictReader(open(mp)):
            acc[short(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
        for k, cs in acc.items():
            busy, gui = cs.get('SQ_VALU_MFMA_BUSY_CYCLES'), cs.get('GRBM_GUI_ACTIVE')
            if not busy or not gui:
                continue
            v = out.setdefault(k, {})
            v['mfma_busy_cycles_avg'] = sum(busy) / len(busy)
            v['grbm_gui_active_avg'] = sum(gui) / len(gui)
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs issue MFMAs
            cyc = v['grbm_gui_active_avg'] / 8
            v['mfma_util'] = v['mfma_busy_cycles_avg'] / (cyc * 1024)
            if v.get('avg_ns'):
                v['clock_ghz'] = cyc / v['avg_ns']
    for k, v in out.items():
        if 'fetch_size_kib_avg' in v and 'write_size_kib_avg' in v:
            v['hbm_read_bytes_corrected'] = 2 * v['fetch_size_kib_avg'] * 1024
            v['hbm_write_bytes'] = v['write_size_kib_avg'] * 1024
            v['hbm_bytes_corrected'] = v['hbm_read_bytes_corrected'] + v['hbm_write_bytes']
    os.makedirs('profiles', exist_ok=True)
    with open(os.path.join('profiles', '%s_kernel_summary.json' % tag), 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)
    lines = ['| kernel | calls | avg us | % | FETCH KiB (raw) | WRITE KiB | HBM MB (corrected) | MFMA util | clock GHz |',
             '|---|---|---|---|---|---|---|---|---|']
    for k, v in sorted(out.items(), key=lambda kv: -kv[1].get('pct', 0)):
        lines.append('| %s | %s | %.1f | %.2f | %s | %s | %s | %s | %s |' % (
            k, v.get('calls', ''), v.get('avg_ns', 0) / 1e3, v.get('pct', 0),
            '%.0f' % v['fetch_size_kib_avg'] if 'fetch_size_kib_avg' in v else '',
            '%.0f' % v['write_size_kib_avg'] if 'write_size_kib_avg' in v else '',
            '%.1f' % (v['hbm_bytes_corrected'] / 1e6) if 'hbm_bytes_corrected' in v else '',
            '%.3f' % v['mfma_util'] if v.get('mfma_busy_cycles_avg') else '',
            '%.2f' % v['clock_ghz'] if v.get('clock_ghz') else ''))
    with open(os.path.join('profiles', '%s_kernel_summary.md' % tag), 'w') as f:
        f.write('\n'.join(lines) + '\n')
    print('\n'.join(lines))


def merge(tags, out_tag):
    """profiles/<out_tag>_kernel_summary.json = the union of several runs'
    summaries (earlier tags win for kernels present in more than one)."""
    out = {}
    for t in reversed(tags):
        with open(os.path.join('profiles', '%s_kernel_summary.json' % t)) as f:
            out.update(json.load(f))
    with open(os.path.join('profiles', '%s_kernel_summary.json' % out_tag), 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    if sys.argv[1] == 'merge':     # python tools/pmc_summary.py merge OUT TAG1 TAG2 ...
        merge(sys.argv[3:], sys.argv[2])
    else:
        main(sys.argv[1], sys.argv[2])
