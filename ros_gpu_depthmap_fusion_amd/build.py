"""Build libgdf.so (HIP, gfx950) in-tree with hipcc."""
from __future__ import annotations

import hashlib
import os
import socket
import subprocess
import time

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_PATH = os.path.join(PKG, "lib", "libgdf.so")
SOURCES = ["gdf_kernels.hip", "gdf_segment.hip", "gdf_engine.cpp", "gdf_driver.cpp",
           "gdf_fused.cpp"]
HEADERS = ["gdf_device.hpp", "gdf_kernels.hpp", "gdf_voxsum.hpp"]

# Float contract of SURVEY.md Appendix A: no FMA contraction, correctly rounded / and sqrt.
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
               "-Wall", "-Wno-unused-result"]


def _deps():
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps += [os.path.join(ROOT, "include", h) for h in ("gdf.h", "gdf_driver.h", "gdf_segment.h", "gdf_fused.h")]
    return deps


def source_digest():
    """sha256 (16 hex digits) of the library's sources, headers and compile flags; None when the
    sources are not present."""
    h = hashlib.sha256()
    for d in _deps():
        if not os.path.exists(d):
            return None
        h.update(os.path.basename(d).encode() + b"\0")
        h.update(open(d, "rb").read())
    h.update(" ".join(HIPCC_FLAGS).encode())
    return h.hexdigest()[:16]


def _stale(out: str, digest) -> bool:
    """The library is rebuilt unless its sidecar stamp names the current source digest (content,
    not mtimes: a copied tree keeps a valid library, an edited one never reuses a stale one)."""
    if not os.path.exists(out) or digest is None:
        return not os.path.exists(out)
    try:
        return open(out + ".sha").read().strip() != digest
    except OSError:
        return True


TRACE_LIB_PATH = os.path.join(PKG, "lib", "libgdf_trace.so")


def build_library(force: bool = False, verbose: bool = False, trace: bool = False) -> str:
    """libgdf.so; trace=True: the diagnostic variant libgdf_trace.so (-DGDF_TRACE_GROUPS: per-group
    timings of the voxel-sum kernel, read by tools/group_trace.py - never the product library)."""
    out = TRACE_LIB_PATH if trace else LIB_PATH
    digest = source_digest()
    if not force and not _stale(out, digest):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    stamp = "source_sha=%s;built_on=%s;built_at=%s" % (
        digest, socket.gethostname(), time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
    cmd = [hipcc, *HIPCC_FLAGS, *(["-DGDF_TRACE_GROUPS"] if trace else []),
           '-DGDF_BUILD_INFO="%s"' % stamp,
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
           "-o", out + ".tmp", *[os.path.join(CSRC, f) for f in SOURCES], "-ldl"]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + r.stdout + r.stderr)
    os.replace(out + ".tmp", out)
    with open(out + ".sha", "w") as f:
        f.write(str(digest) + "\n")
    return out
