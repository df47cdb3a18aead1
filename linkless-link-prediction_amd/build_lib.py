"""Build libllp_hip.so in-tree (gfx950 only): ``python build_lib.py [--force]``.

Each csrc/*.hip / *.cpp is compiled by hipcc with --offload-arch=gfx950 into
csrc/build/*.o, then linked into ``libllp_hip.so`` next to this file.  Objects
are rebuilt only when their source or a header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libllp_hip.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I", INCLUDE, "-I", CSRC,
         "-Wno-unused-result", "-munsafe-fp-atomics"]


def _newest_header():
    hs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _compile(src, obj, force, extra=()):
    if not force and os.path.exists(obj):
        if os.path.getmtime(obj) >= max(os.path.getmtime(src), _newest_header()):
            return obj, None
    cmd = [HIPCC, *FLAGS, *extra, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(os.path.join(CSRC, "build"), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    objs = [os.path.join(CSRC, "build", os.path.basename(s) + ".o") for s in srcs]
    return _build(srcs, objs, OUT, force, verbose, [])


def build_variant(out: str, defines, sources=("dedup.hip",), verbose: bool = True) -> str:
    """An A/B build of the library at ``out``: ``sources`` compiled with the extra
    ``-D`` ``defines`` (objects under csrc/build/<tag>/), every other object shared
    with the default build.  Used by tools/ for same-box comparisons (LLP_LIB)."""
    build(verbose=False)
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    tag = os.path.splitext(os.path.basename(out))[0]
    os.makedirs(os.path.join(CSRC, "build", tag), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    objs = [os.path.join(CSRC, "build", tag if os.path.basename(s) in sources else "", os.path.basename(s) + ".o")
            for s in srcs]
    return _build(srcs, objs, out, False, verbose, ["-D" + d for d in defines],
                  only={os.path.basename(s) for s in srcs if os.path.basename(s) in sources})


def _build(srcs, objs, out, force, verbose, extra, only=None):
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    todo = [(s, o) for s, o in zip(srcs, objs) if only is None or os.path.basename(s) in only]
    with cf.ThreadPoolExecutor(max_workers=max(jobs, 1)) as ex:
        results = list(ex.map(lambda so: _compile(so[0], so[1], force, extra), todo))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("libllp_hip build failed:\n" + "\n".join(errs))
    if force or not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", *objs, "-o", out]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"built {out}")
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
