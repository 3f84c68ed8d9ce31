"""germline_direct timing on the bench shard (configs[1]: chr20 length, 30x), one process per
GQ_DBG setting (read once per process): the pileup kernel's HIP-event time per call and, with
GQ_DBG=16, its phase clocks (cycles per tile and wave, printed by the library on stderr).
usage: python scripts/direct_ablate.py [length]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(L):
    sys.path.insert(0, ROOT)
    import numpy as np
    from guacamole_amd import native, synthetic
    g = synthetic.generate(L, 30.0, seed=synthetic.SEED + 2)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([L - 1], np.int64), np.array([0], np.int64))
    ctx = native.Context(0)
    reads = ctx.upload(g.arrays)
    ms = []
    for k in range(6):
        ctx.rederive(reads)
        ctx.germline_threshold_device(reads, loci, 8)
        tm = ctx.timings()
        if k >= 2:
            ms.append(tm["pileup_ms"])
    print("GQ_DBG=%s pileup_ms median %.3f (walk_tiles %d)" % (os.environ.get("GQ_DBG", "0"), float(np.median(ms)),
                                                               tm["walk_tiles"]), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "child":
        child(int(sys.argv[1]))
        sys.exit(0)
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 63025520
    for dbg in os.environ.get("DBGS", "0 16 1 4 5").split():
        env = dict(os.environ, GQ_DBG=dbg)
        r = subprocess.run([sys.executable, __file__, str(L), "child"], env=env, capture_output=True, text=True,
                           timeout=300)
        print(r.stdout.strip(), "|", " ".join(l for l in r.stderr.splitlines() if "prof" in l)[-300:], flush=True)
        if r.returncode != 0:
            print(r.stderr[-2000:])
            sys.exit(r.returncode)
