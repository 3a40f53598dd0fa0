"""In-tree builds of the native libraries (no JIT cache: the .so files travel with
the repo snapshot to the GPU box).

  libmpc.so        HIP kernels + C-ABI (include/mpc.h), hipcc --offload-arch=gfx950
  libmpc_synth.so  host-only synthetic data generator (g++)
  libmpc_ingest.so native host I/O: ingest (Steps 1-3) and writers (Step 7) (include/mpc_ingest.h, g++ -pthread)
"""
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIBMPC = os.path.join(PKG, "libmpc.so")
LIBSYNTH = os.path.join(PKG, "libmpc_synth.so")
LIBINGEST = os.path.join(PKG, "libmpc_ingest.so")

HIP_SOURCES = ["mpc_kernels.hip"]
HIP_HEADERS = ["mpc_device.h"]


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.exists(s) and os.path.getmtime(s) > t for s in sources)


def build_synth(force=False):
    src = os.path.join(CSRC, "synth.cpp")
    if force or _stale(LIBSYNTH, [src, os.path.join(CSRC, "host_threads.h")]):
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", LIBSYNTH, src], check=True)
    return LIBSYNTH


def ensure_synth():
    return build_synth()


def build_ingest(force=False):
    srcs = [os.path.join(CSRC, f) for f in ("ingest.cpp", "writers.cpp", "pseudopair.cpp")]
    hdr = os.path.join(INCLUDE, "mpc_ingest.h")
    if force or _stale(LIBINGEST, srcs + [hdr, os.path.join(CSRC, "host_threads.h")]):
        subprocess.run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-I", INCLUDE, "-o", LIBINGEST] + srcs,
                       check=True)
    return LIBINGEST


def build_hip(force=False, extra=(), out=None):
    """libmpc.so (``out``/``extra``: experiment variants, e.g. -DMPC_TUNING_OVERRIDES)."""
    out = out or LIBMPC
    srcs = [os.path.join(CSRC, s) for s in HIP_SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in HIP_HEADERS] + [os.path.join(INCLUDE, "mpc.h")]
    if force or extra or _stale(out, deps):
        hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
        cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-I", INCLUDE, "-I", CSRC, "-o", out] + list(extra) + srcs
        subprocess.run(cmd, check=True)
    return out


def build_all(force=False):
    build_synth(force)
    build_ingest(force)
    build_hip(force)
