"""Codegen inspection: list the loops (backward branches) of a gfx950 assembly file with their
instruction counts, LDS/global traffic, waits and spill traffic.

    make -C learning-based-mpc_amd isa && python tools/isa_loops.py [file.s] [--dump START END]
"""
import collections
import re
import sys


def main():
    args = sys.argv[1:]
    path = args[0] if args and not args[0].startswith('--') else \
        'learning-based-mpc_amd/build/isa/ocp_mg10.s'
    lines = open(path).read().split('\n')
    if '--dump' in args:
        i = args.index('--dump')
        a, b = int(args[i + 1]), int(args[i + 2])
        for n in range(a, b + 1):
            ln = lines[n - 1]
            if ln.strip() and not ln.strip().startswith(';') and not ln.strip().startswith('.'):
                print(n, ln)
        return
    if '--phases' in args:
        phases(lines)
        return
    pos = {}
    loops = []
    for n, ln in enumerate(lines, 1):
        m = re.match(r'^(\.LBB[0-9_]+):', ln)
        if m:
            pos[m.group(1)] = n
        m = re.match(r'^\s+s_(cbranch_\w+|branch)\s+(\.LBB[0-9_]+)', ln)
        if m and m.group(2) in pos:
            loops.append((pos[m.group(2)], n))
    ins = re.compile(r'^\s+([vsdgb][a-z_0-9]+)')
    for a, b in sorted(set(loops)):
        c = collections.Counter()
        for ln in lines[a - 1:b]:
            m = ins.match(ln)
            if m:
                c[m.group(1)] += 1
        tot = sum(c.values())
        key = lambda p: sum(v for k, v in c.items() if k.startswith(p))
        print('%6d-%6d  instr %5d  fma %4d  ds_r %3d  ds_w %3d  glob %3d  wait %3d  rdlane %3d  agpr %3d  div %2d  scratch %2d'
              % (a, b, tot, key('v_fma') + key('v_fmac'), key('ds_read'), key('ds_write'),
                 key('global_'), key('s_waitcnt'), key('v_readlane'), key('v_accvgpr'),
                 c['v_div_fixup_f64'], key('scratch_')))


NAMES = {0: 'residuals', 1: 'factor:recip+Dx', 2: "factor:F'DF", 3: 'factor:riccati',
         4: "solve:q+F'e", 5: 'solve:prepass', 6: 'solve:backward', 7: 'solve:post-bwd',
         8: 'solve:forward', 9: 'solve:post-fwd', 10: 'step_len', 11: 'comp_after',
         12: 'row update', 13: 'stage update', 14: 'loop top', 15: 'solve start'}


def phases(lines):
    """Static instruction mix between consecutive ;BQP_PHASE markers (ISA build).  STAMP(id)
    closes phase id, so a region is named after the marker that ENDS it."""
    ins = re.compile(r'^\s+([vsdgb][a-z_0-9]+)')
    cur, c, start = None, collections.Counter(), 0
    out = []
    for n, ln in enumerate(lines, 1):
        m = re.search(r';BQP_PHASE (\d+)', ln)
        if m:
            if cur is not None:
                out.append((start, int(m.group(1)), c))
            cur, c, start = int(m.group(1)), collections.Counter(), n
            continue
        m = ins.match(ln)
        if m and cur is not None:
            c[m.group(1)] += 1
    for start, ph, c in out:
        key = lambda p: sum(v for k, v in c.items() if k.startswith(p))
        print('%6d  ->%-16s instr %5d  fma %4d  ds_r %3d  ds_w %3d  wait %3d  rdlane %3d  agpr %3d  dpp %3d  div %2d'
              % (start, NAMES.get(ph, ph), sum(c.values()), key('v_fma') + key('v_fmac'), key('ds_read'),
                 key('ds_write'), key('s_waitcnt'), key('v_readlane'), key('v_accvgpr'),
                 key('v_mov_b32_dpp'), c['v_div_fixup_f64']))


if __name__ == '__main__':
    main()
