"""In-tree build of libcnf_hip.so (hipcc, gfx950). The .so is git-ignored but travels
to the GPU box with the repository snapshot."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / 'csrc'
# CNF_BUILD_LIB: write a diagnostic build elsewhere (e.g. the host-sanitizer build, tools/host_sanitize.sh)
LIB = Path(os.environ['CNF_BUILD_LIB']) if os.environ.get('CNF_BUILD_LIB') else PKG / 'lib' / 'libcnf_hip.so'
SOURCES = ['cnf_kernels.hip', 'cnf_stream.hip', 'cnf_netlds.hip', 'cnf_toy.hip', 'cnf_train.hip', 'cnf_ldsbwd.hip', 'cnf_transforms.hip', 'cnf_runtime.cpp',
           'cnf_plan.cpp', 'cnf_train.cpp', 'cnf_comm.cpp']
HEADERS = ["cnf_kernels.h", "cnf_device.h", "cnf_plan.h", "cnf_netlds_shapes.inc", "cnf_gc_shapes.inc", "cnf_pw_shapes.inc"]
ARCH = os.environ.get('CNF_OFFLOAD_ARCH', 'gfx950')


def _hipcc() -> str:
    for cand in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', 'hipcc'):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError('hipcc not found')


def _extra_flags() -> list:
    return os.environ.get('CNF_EXTRA_FLAGS', '').split()   # diagnostics, e.g. -DCNF_GC_STAMPS


def _flags_file() -> Path:
    return LIB.with_suffix('.so.flags')


def _objdir() -> Path:
    """Objects live in a directory per flag set, so a diagnostic build (CNF_EXTRA_FLAGS) never
    leaves instrumented objects for a later normal build to reuse."""
    import hashlib
    fl = ' '.join(_extra_flags())
    return PKG / 'build' / ('default' if not fl else 'x' + hashlib.sha1(fl.encode()).hexdigest()[:12])


def needs_build() -> bool:
    if not LIB.exists():
        return True
    ff = _flags_file()
    built_with = ff.read_text() if ff.exists() else ''
    if built_with != ' '.join(_extra_flags()):
        return True
    t = LIB.stat().st_mtime
    deps = [CSRC / s for s in SOURCES + HEADERS] + [PKG.parent / 'include' / 'cnf.h']
    return any(p.stat().st_mtime > t for p in deps if p.exists())


def _compile(src: Path, obj: Path, verbose: bool) -> None:
    cmd = [_hipcc(), f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-fPIC', '-Wno-pass-failed', '-c',
           '-o', str(obj), str(src)]
    cmd[1:1] = _extra_flags()
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc failed on {src.name} ({r.returncode}):\n{r.stdout}\n{r.stderr}')


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile every translation unit to an object (in parallel, each only when it or a header
    changed), then link libcnf_hip.so."""
    if not force and not needs_build():
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    LIB.parent.mkdir(parents=True, exist_ok=True)
    objdir = _objdir()
    objdir.mkdir(parents=True, exist_ok=True)
    hdr_t = max((CSRC / h).stat().st_mtime for h in HEADERS)
    hdr_t = max(hdr_t, (PKG.parent / 'include' / 'cnf.h').stat().st_mtime)
    jobs = []
    objs = []
    for s in SOURCES:
        src, obj = CSRC / s, objdir / (s + '.o')
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_t):
            jobs.append((src, obj))
    workers = max(1, min(len(jobs), int(os.environ.get('MAX_JOBS', os.cpu_count() or 4)), 8))
    with ThreadPoolExecutor(workers) as ex:
        for f in [ex.submit(_compile, src, obj, verbose) for src, obj in jobs]:
            f.result()
    tmp = LIB.with_suffix('.so.tmp')
    cmd = ([_hipcc(), f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', str(tmp)] + [str(o) for o in objs] + ['-ldl']
           + os.environ.get('CNF_EXTRA_LDFLAGS', '').split())
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'link failed ({r.returncode}):\n{r.stdout}\n{r.stderr}')
    os.replace(tmp, LIB)
    _flags_file().write_text(' '.join(_extra_flags()))
    return LIB


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
