"""Register / LDS / spill figures of librod.so's gfx950 kernels (CPU only: the code object is
unbundled into a temporary directory with llvm-objdump --offloading, the AMDGPU metadata notes
read with llvm-readelf).  usage: python tools/kstats.py <substring> [<substring> ...]"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = '/opt/rocm/lib/llvm/bin'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd', 'lib', 'librod.so')


def kernels():
    with tempfile.TemporaryDirectory() as tmp:
        so = os.path.join(tmp, 'librod.so')
        shutil.copy(LIB, so)
        subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '--offloading', so], cwd=tmp, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        out = []
        for f in sorted(os.listdir(tmp)):
            if not f.endswith('gfx950'):
                continue
            notes = subprocess.run([os.path.join(LLVM, 'llvm-readelf'), '--notes', os.path.join(tmp, f)],
                                   check=True, capture_output=True, text=True).stdout
            # one metadata map per kernel: split at each '.name:' and read the fields around it
            for block in re.split(r'\n\s+- \.agpr_count:', notes)[1:]:
                d = {}
                for key in ('name', 'vgpr_count', 'sgpr_count', 'vgpr_spill_count', 'sgpr_spill_count',
                            'group_segment_fixed_size', 'private_segment_fixed_size', 'agpr_count'):
                    m = re.search(r'\.%s:\s+(\S+)' % key, block)
                    if m:
                        d[key] = m.group(1)
                m = re.match(r'\s*(\d+)', block)
                if m:
                    d['agpr_count'] = m.group(1)
                if 'name' in d:
                    out.append(d)
        return out


def main():
    pats = sys.argv[1:] or ['']
    dem = {}
    ks = kernels()
    names = [k['name'] for k in ks]
    r = subprocess.run(['c++filt'], input='\n'.join(names), capture_output=True, text=True)
    for n, d in zip(names, r.stdout.splitlines()):
        dem[n] = d
    for k in ks:
        d = dem.get(k['name'], k['name'])
        if any(p in d or p in k['name'] for p in pats):
            print('vgpr %4s agpr %3s spill %3s/%-3s lds %6s scratch %5s  %s' % (
                k.get('vgpr_count'), k.get('agpr_count'), k.get('vgpr_spill_count'), k.get('sgpr_spill_count'),
                k.get('group_segment_fixed_size'), k.get('private_segment_fixed_size'), d[:150]))


if __name__ == '__main__':
    main()
