"""Per-launch HBM bytes of the solve kernel from rocprofv3 PMC passes (tools/gpu_prof.sh).

    python tools/pmc_summary.py gpurun_out/TAG profiles/rNN_TAG [--kernel ocp_ipm_kernel] [--config C2]

Reads TAG/pmc_fetch/run_counter_collection.csv (FETCH_SIZE, KB) and TAG/pmc_write/... (WRITE_SIZE,
KB), keeps the dispatches of the named kernel, and applies the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts half the bytes of a wide
read (x2); WRITE_SIZE is taken as is.  Writes OUT/pmc.json and, with --config NAME,
profiles/pmc_NAME.json (read by bench.py as roofline.traffic of that config's line), and copies
the kernel-trace stats + PMC csvs into OUT.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path, kernel):
    out = []
    for r in csv.DictReader(open(path)):
        if kernel in r['Kernel_Name']:
            out.append(r)
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    kernel = 'ocp_ipm_kernel'
    if '--kernel' in sys.argv:
        kernel = sys.argv[sys.argv.index('--kernel') + 1]
    os.makedirs(dst, exist_ok=True)
    fr = rows(os.path.join(src, 'pmc_fetch', 'run_counter_collection.csv'), kernel)
    wr = rows(os.path.join(src, 'pmc_write', 'run_counter_collection.csv'), kernel)
    fetch = [float(r['Counter_Value']) * 1024 for r in fr if r['Counter_Name'] == 'FETCH_SIZE']
    write = [float(r['Counter_Value']) * 1024 for r in wr if r['Counter_Name'] == 'WRITE_SIZE']
    f_b = 2.0 * sum(fetch) / len(fetch)
    w_b = sum(write) / len(write)
    r0 = fr[0]
    res = {
        'kernel': r0['Kernel_Name'], 'grid': int(r0['Grid_Size']),
        'workgroup': int(r0['Workgroup_Size']), 'scratch_bytes_per_lane': int(r0['Scratch_Size']),
        'vgpr': int(r0['VGPR_Count']), 'launches': [len(fetch), len(write)],
        'fetch_bytes_per_launch': f_b, 'write_bytes_per_launch': w_b,
        'hbm_bytes_per_launch': f_b + w_b,
        'correction': 'FETCH_SIZE x 1024 x 2 (gfx950: half of wide reads counted), '
                      'WRITE_SIZE x 1024; separate --pmc passes',
    }
    ks = os.path.join(src, 'trace', 'run_kernel_stats.csv')
    if os.path.exists(ks):      # rocprofv3 --stats average of the same kernel (kernel-trace pass)
        for r in csv.DictReader(open(ks)):
            if kernel in r.get('Name', ''):
                res['trace_avg_ms'] = float(r['AverageNs']) * 1e-6
                res['trace_calls'] = int(r['Calls'])
                break
    json.dump(res, open(os.path.join(dst, 'pmc.json'), 'w'), indent=1)
    res['source'] = dst
    if '--config' in sys.argv:
        name = sys.argv[sys.argv.index('--config') + 1]
        json.dump(res, open(os.path.join(ROOT, 'profiles', 'pmc_%s.json' % name), 'w'), indent=1)
    for sub, name in (('trace', 'run_kernel_stats.csv'), ('pmc_fetch', 'run_counter_collection.csv'),
                      ('pmc_write', 'run_counter_collection.csv')):
        p = os.path.join(src, sub, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, '%s_%s' % (sub, name)))
    for log in ('bench.log', 'bench_trace.log', 'stamps.log', 'stamps.json', 'pytest_gpu.log'):
        p = os.path.join(src, log)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, log))
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
