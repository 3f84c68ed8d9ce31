#!/usr/bin/env python3
"""The bench's measured single pass (germline-threshold CLI on the configs[1] shard written as
a BAM), once per ingest mode: GQ_INGEST=device (BAM decoded on the GPU) and host.
  python scripts/single_pass.py [--length L] [--modes device,host]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from guacamole_amd import synthetic
    ap = argparse.ArgumentParser()
    ap.add_argument("--length", type=int, default=bench.CHR20)
    ap.add_argument("--modes", default="device,host")
    a = ap.parse_args()
    g = synthetic.generate(a.length, 30.0)
    for mode in a.modes.split(","):
        os.environ["GQ_INGEST"] = mode
        r = bench.single_pass(g, a.length)
        print(json.dumps(dict(mode=mode, **r)), flush=True)


if __name__ == "__main__":
    main()
