"""Build helpers: compile the HIP library in-tree for gfx950 (hipcc) and the
test oracle (g++).  Used by __graft_entry__.build()."""
from __future__ import annotations

import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "guacamole_amd")
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "_lib")
LIB = os.path.join(LIB_DIR, "libgqpileup.so")
SOURCES = [os.path.join(CSRC, f) for f in ("gq_pileup.hip", "gq_somatic.hip", "gq_heapref.hip", "gq_bamdev.hip")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + [
    os.path.join(ROOT, "include", "gqpileup.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GQ_OFFLOAD_ARCH", "gfx950")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_hip(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    if force or _stale(LIB, DEPS):
        # one hipcc per translation unit, in parallel, then one link
        objs = [os.path.join(LIB_DIR, os.path.basename(s) + ".o") for s in SOURCES]
        procs = []
        for src, obj in zip(SOURCES, objs):
            cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-c",
                   "-I" + os.path.join(ROOT, "include"), "-o", obj, src]
            if verbose:
                print(" ".join(cmd))
            procs.append((cmd, subprocess.Popen(cmd)))
        for cmd, p in procs:
            if p.wait() != 0:
                raise subprocess.CalledProcessError(p.returncode, cmd)
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs + ["-lz"]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
        for obj in objs:
            os.remove(obj)
    return LIB


SYNTH_SRC = os.path.join(CSRC, "gq_synth.cpp")
SYNTH_LIB = os.path.join(LIB_DIR, "libgqsynth.so")


def build_synth(force: bool = False) -> str:
    """Host-side synthetic read generator (bench / test data), g++ -O3 -pthread."""
    os.makedirs(LIB_DIR, exist_ok=True)
    if force or _stale(SYNTH_LIB, [SYNTH_SRC]):
        subprocess.check_call(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", SYNTH_LIB, SYNTH_SRC,
                               "-lz"])
    return SYNTH_LIB


INGEST_SRC = os.path.join(CSRC, "gq_ingest.cpp")
INGEST_LIB = os.path.join(LIB_DIR, "libgqingest.so")


def build_ingest(force: bool = False) -> str:
    """Host read ingest (BGZF/BAM decode, MD events), g++ -O3 -pthread, zlib."""
    os.makedirs(LIB_DIR, exist_ok=True)
    if force or _stale(INGEST_LIB, [INGEST_SRC, os.path.join(ROOT, "include", "gqingest.h")]):
        subprocess.check_call(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", INGEST_LIB,
                               INGEST_SRC, "-lz", "-ldl"])
    return INGEST_LIB


def build_oracle() -> str:
    d = os.path.join(ROOT, "oracle")
    subprocess.check_call(["make", "-s", "-C", d])
    return os.path.join(d, "_build", "liboracle.so")
