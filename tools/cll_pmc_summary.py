"""Summarise the CLL profile passes of tools/gpu_r04_final.sh / gpu_r04_prof.sh (dense sub-problem
kernel: HBM bytes per launch with the gfx950 FETCH_SIZE correction, MFMA busy cycles, trace average)
into OUT/pmc.json and profiles/pmc_CLL.json (read by bench.py's CLL roofline).
Usage: python tools/cll_pmc_summary.py gpurun_out/TAG/CLL profiles/TAG/CLL"""
import collections
import csv
import json
import os
import shutil
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)

    def avg(pas, cname, kern='dense_ipm_kernel'):
        v = [float(r['Counter_Value']) for r in csv.DictReader(open(os.path.join(src, pas, 'run_counter_collection.csv')))
             if kern in r['Kernel_Name'] and r['Counter_Name'] == cname]
        return sum(v) / len(v), len(v)
    f, nf = avg('pmc_fetch', 'FETCH_SIZE')
    w, nw = avg('pmc_write', 'WRITE_SIZE')
    mb, _ = avg('pmc_mfma', 'SQ_VALU_MFMA_BUSY_CYCLES')
    gg, _ = avg('pmc_mfma', 'GRBM_GUI_ACTIVE')
    sb, _ = avg('pmc_mfma', 'SQ_BUSY_CYCLES')
    st = [r for r in csv.DictReader(open(os.path.join(src, 'trace', 'run_kernel_stats.csv')))
          if 'dense_ipm_kernel' in r['Name']][0]
    res = {'kernel': 'dense_ipm_kernel<true> (learned-model loop sub-problem, n = 101, m = 1024, batch 256)',
           'fetch_bytes_per_launch': 2 * f * 1024, 'write_bytes_per_launch': w * 1024,
           'hbm_bytes_per_launch': 2 * f * 1024 + w * 1024, 'launches': [nf, nw],
           'sq_valu_mfma_busy_cycles': mb, 'grbm_gui_active': gg, 'sq_busy_cycles': sb,
           'mfma_busy_frac_est': mb / (gg / 8 * 1024),
           'trace_avg_ms': float(st['AverageNs']) * 1e-6, 'trace_calls': int(st['Calls']),
           'correction': 'FETCH_SIZE x 1024 x 2 (gfx950), WRITE_SIZE x 1024; separate --pmc passes; '
                         'mfma_busy_frac_est = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)',
           'source': dst}
    json.dump(res, open(os.path.join(dst, 'pmc.json'), 'w'), indent=1)
    json.dump(res, open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles',
                                      'pmc_CLL.json'), 'w'), indent=1)
    shutil.copy(os.path.join(src, 'trace', 'run_kernel_stats.csv'), os.path.join(dst, 'trace_run_kernel_stats.csv'))
    for pas in ('pmc_mfma', 'pmc_fetch', 'pmc_write'):
        shutil.copy(os.path.join(src, pas, 'run_counter_collection.csv'), os.path.join(dst, pas + '_run_counter_collection.csv'))
    print(json.dumps(res))


if __name__ == '__main__':
    main()
