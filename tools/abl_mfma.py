"""Timing ablation (diagnostic, wrong results): a build of the library in which every forward MFMA
k-step with an odd index is skipped, i.e. half of the fp32 MFMA issue of k_net_lds, k_pw and k_gc.
It bounds what a cheaper contraction (e.g. a bf16x3 split at 0.375x the fp32 MFMA cycles) can win
per kernel before any of it is written. Output: arl_conditional_normalizing_flows_amd/lib/libcnf_abl.so
(load it with CNF_LIB=... bench.py --no-cpu-baseline)."""
import os
import re
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / 'arl_conditional_normalizing_flows_amd'
sys.path.insert(0, str(ROOT))
from arl_conditional_normalizing_flows_amd import _build  # noqa: E402

OUT = PKG / 'lib' / 'libcnf_abl.so'
MF = '__builtin_amdgcn_mfma_f32_16x16x4f32'


def ablate(txt: str) -> str:
    # unrolled k-step sites: acc = MF(x[.. s ..], ...) -> acc = (s & 1) ? acc : MF(...)
    pat = re.compile(r'(\b[\w\[\]]+) = ' + MF + r'\(([^;]*?\[(s4|s|q)\][^;]*)\);')
    txt, n1 = pat.subn(lambda m: f'{m.group(1)} = ({m.group(3)} & 1) ? {m.group(1)} : {MF}({m.group(2)});', txt)
    # PK_KN k0 loops
    pat2 = re.compile(r'(\b[\w\[\]]+) = ' + MF + r'\((a[01]), ([^;]*?)\);')
    txt, n2 = pat2.subn(lambda m: f'{m.group(1)} = ((k0 >> 2) & 1) ? {m.group(1)} : {MF}({m.group(2)}, {m.group(3)});', txt)
    return txt, n1 + n2


def main():
    tmp = Path(tempfile.mkdtemp(prefix='cnf_abl_'))
    src = tmp / 'pkg' / 'csrc'   # (csrc/../../include/cnf.h)
    shutil.copytree(PKG / 'csrc', src)
    (tmp / 'include').mkdir()
    shutil.copy(ROOT / 'include' / 'cnf.h', tmp / 'include' / 'cnf.h')
    tot = 0
    for f in ('cnf_netlds.hip', 'cnf_stream.hip'):
        t, n = ablate((src / f).read_text())
        (src / f).write_text(t)
        print(f, n, 'sites')
        tot += n
    objs = []
    jobs = []
    for s in _build.SOURCES:
        if s in ('cnf_netlds.hip', 'cnf_stream.hip'):
            o = tmp / (s + '.o')
            jobs.append((src / s, o))
        else:
            o = _build._objdir() / (s + '.o')   # the default build's objects
        objs.append(o)
    with ThreadPoolExecutor(8) as ex:
        for fut in [ex.submit(_build._compile, a, b, False) for a, b in jobs]:
            fut.result()
    cmd = [_build._hipcc(), '--offload-arch=gfx950', '-shared', '-fPIC', '-o', str(OUT)] + [str(o) for o in objs] + ['-ldl']
    subprocess.run(cmd, check=True)
    print(OUT, tot)


if __name__ == '__main__':
    main()
