"""Build libhbx.so (all HIP kernels + the C ABI) for gfx950, in-tree.

    python -m hpbandster_amd.build [--force] [--jobs N]

Each .hip/.cpp file in hpbandster_amd/csrc is compiled with hipcc --offload-arch=gfx950 into an
object under hpbandster_amd/_lib/obj, then linked into hpbandster_amd/_lib/libhbx.so.  Objects
are rebuilt only when their source or a header is newer.  No torch extension machinery: the
library exposes a plain extern "C" ABI (include/hbx.h) loaded with ctypes.
"""

import argparse
import concurrent.futures
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(os.path.dirname(PKG), "include")
LIBDIR = os.path.join(PKG, "_lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libhbx.so")
ARCH = os.environ.get("HBX_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libhbx.so)")


def _flags():
    return ["-O3", "-std=c++17", "-fPIC", "--offload-arch=%s" % ARCH, "-I", CSRC, "-I", INCLUDE,
            "-Wno-unused-result", "-munsafe-fp-atomics",
            # bit-exact fp64 paths (np.std, the exact re-score) must not be contracted into FMAs;
            # the fp32 scoring kernel spells its FMAs out with fmaf()
            "-ffp-contract=off"]


# per-file extra flags: the scoring loops interleave MFMAs with scalar f32 adds; SLP packing them into
# v_pk_add_f32 costs more issue cycles beside MFMAs than the plain adds (MI355X_MICROARCH.md)
EXTRA_FLAGS = {"hbx_score_h.hip": ["-fno-slp-vectorize"], "hbx_score_h32.hip": ["-fno-slp-vectorize"], "hbx_score_oh.hip": ["-fno-slp-vectorize"],
               "hbx_score_f32.hip": ["-fno-slp-vectorize"]}


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _newest_header():
    hs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _compile(src, force):
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), _newest_header()):
        return obj, False
    cmd = [hipcc()] + _flags() + EXTRA_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s" % (src, r.stdout))
    return obj, True


def build(force=False, jobs=None, verbose=True):
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sources()
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 2) // 2), 8)
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force), srcs))
    objs = [o for o, _ in results]
    rebuilt = any(r for _, r in results)
    if rebuilt or force or not os.path.exists(LIB):
        tmp = LIB + ".tmp"
        # RCCL for the multi-GPU winner exchange (hbx_dist.hip); at run time the SONAME librccl.so.1
        # resolves to the copy torch has already loaded, so one RCCL runtime serves both
        cmd = [hipcc(), "-shared", "-fPIC", "--offload-arch=%s" % ARCH, "-o", tmp] + objs + [
            "-L/opt/rocm/lib", "-lrccl"]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s" % r.stdout)
        os.replace(tmp, LIB)
        if verbose:
            print("built %s (%d objects)" % (LIB, len(objs)))
    elif verbose:
        print("%s is up to date" % LIB)
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    sys.exit(main())
