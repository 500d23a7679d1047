"""Per-kernel VGPR / AGPR / scratch / LDS of the gfx950 code objects inside a built library or
object (the clang offload bundles of the .hip_fatbin section), from the AMDGPU metadata notes.
Usage: python tools/kres.py learning-based-mpc_amd/bqp/libbqp.so [name-filter]"""
import re
import struct
import subprocess
import sys
import tempfile

B = '/opt/rocm/llvm/bin'
MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'


def bundles(data):
    pos = 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return
        n = struct.unpack_from('<Q', data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from('<QQQ', data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if 'gfx950' in triple:
                yield data[i + off:i + off + size]
        pos = i + 1


def main():
    data = open(sys.argv[1], 'rb').read()
    flt = sys.argv[2] if len(sys.argv) > 2 else ''
    for co in bundles(data):
        with tempfile.NamedTemporaryFile(suffix='.co') as f:
            f.write(co)
            f.flush()
            out = subprocess.run([B + '/llvm-readelf', '--notes', f.name], capture_output=True, text=True).stdout
        for blk in re.split(r'\n  - ', out):
            m = re.search(r'\.name:\s+(\S+)', blk)
            if not m or flt not in m.group(1):
                continue
            dm = subprocess.run(['c++filt'], input=m.group(1), capture_output=True, text=True).stdout.strip()
            g = lambda k: (re.search(k + r':\s+(\d+)', blk) or [None, '?'])[1]
            print('%-72s vgpr %4s agpr %4s scratch %5s' % (dm[:72], g(r'\.vgpr_count'), g(r'\.agpr_count'),
                                                          g(r'\.private_segment_fixed_size')))


if __name__ == '__main__':
    main()
