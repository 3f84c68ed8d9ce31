"""The library's alternative kernel builds, picked per process from the environment, give the
default build's records bit for bit (the default is checked against the oracle elsewhere):
GQ_CALL_SPLIT=1 (somatic caller as a front kernel + back end over stored element records),
GQ_CALL_WPE=2 (the one-kernel caller at 2 waves per SIMD), GQ_FILL_U=2 / 4 (the read-major
projection and margin fills at 2 or 4 words per lane and round; GQ_FILL_W: 2 or 4 consecutive
words of a read per lane), GQ_FILL_ONE=1 (the projection and the margin projection in one pass
instead of two) — each with GQ_FILL=rw (the read-major fills), GQ_FILL=slice (the slice-major
fills), GQ_ROWS=firstfit (first-fit row assignment instead of the parallel earliest-freed one),
GQ_FILL=pieces (the projection by pieces instead of cells), GQ_MFILL=cells / pieces (the margin
projection by cells / pieces instead of read-major), GQ_GERM=proj (germline-threshold through
germline_proj over the projection instead of germline_direct straight from the reads; the
projection-fill variants run with it, so their germline records come from the fill under test),
GQ_SOM=proj (somatic-standard's candidates from somatic_proj over the projection and margin
projection instead of somatic_direct; the projection and margin-fill variants run with it).
A synthetic 300 kb 60x / 30x pair with a raised somatic
rate, so hundreds of candidates and calls reach every path."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra):
    env = dict(os.environ, PYTHONPATH=ROOT, **extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_variant_runner.py"), "300000"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_kernel_variants_give_the_default_records():
    base = _run({})
    assert base["somatic"] > 20 and base["germline"] > 100
    pj = {"GQ_GERM": "proj", "GQ_SOM": "proj"}
    rw = dict(pj, GQ_FILL="rw")
    for extra in ({"GQ_CALL_SPLIT": "1"}, {"GQ_CALL_WPE": "2"}, {"GQ_SOM": "proj"}, pj, rw, dict(rw, GQ_FILL_U="2"),
                  dict(rw, GQ_FILL_U="4"), dict(rw, GQ_FILL_W="2"), dict(rw, GQ_FILL_W="4"), dict(rw, GQ_FILL_ONE="1"),
                  dict(pj, GQ_FILL="slice"), dict(pj, GQ_ROWS="firstfit"), dict(pj, GQ_FILL="pieces"),
                  dict(pj, GQ_FILL="cellsb"), dict(pj, GQ_MFILL="cells"), dict(pj, GQ_MFILL="pieces")):
        got = _run(extra)
        assert got == base, (extra, got, base)
