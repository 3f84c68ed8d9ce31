"""The multi-GPU product path (configs[3] shape) on one GPU: the CLI launched by
torch.distributed.run with two ranks (gloo gather, both ranks on cuda:0) writes exactly what the
single-process run with the same task partition writes.  Cuts between the ranks fall inside
chrM's 150x coverage, so reads straddling them go to both ranks (DistributedUtil.scala:584-597)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import fixture

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, world, out, reports=None, extra_env=None):
    """The CLI at `world` ranks; reports: a list that receives each rank's GQ_TIMING report."""
    env = dict(os.environ, GQ_DIST_BACKEND="gloo", PYTHONPATH=ROOT, GQ_TIMING="1", **(extra_env or {}))
    if world == 1:
        cmd = [sys.executable, "-m", "guacamole_amd"] + args + ["--out", out]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "guacamole_amd"] + args + ["--out", out]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    if reports is not None:
        import json
        for line in r.stderr.splitlines():
            if "GQ_TIMING " in line:
                reports.append(json.loads(line.split("GQ_TIMING ", 1)[1]))
    with open(out) as fh:
        return fh.read()


@pytest.mark.parametrize("parallelism", ["2", "5"])
def test_germline_two_ranks_equal_one(tmp_path, parallelism):
    args = ["germline-threshold", "--reads", fixture("chrM.sorted.bam"), "--parallelism", parallelism,
            "--partition-accuracy", "0"]
    one = _run(args, 1, str(tmp_path / "one.json"))
    two = _run(args, 2, str(tmp_path / "two.json"))
    assert one == two and one.count("\n") > 100


def test_somatic_two_ranks_equal_one(tmp_path):
    args = ["somatic-standard", "--tumor-reads", fixture("tumor.chr20.tough.sam"), "--normal-reads",
            fixture("normal.chr20.tough.sam"), "--parallelism", "6", "--odds", "2"]
    one = _run(args, 1, str(tmp_path / "one.json"))
    two = _run(args, 2, str(tmp_path / "two.json"))
    assert one == two and one.count("\n") > 10


def _bench(world, out, extra):
    env = dict(os.environ, GQ_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    args = ["bench.py", "--gpus", str(world), "--steps", "1", "--warmup", "0", "--somatic-length", "0", "--panel-length", "0",
            "--no-single-pass", "--no-configs3",
            "--no-cpu-baseline", "--shared-reads", "--calls-out", out] + extra
    if world == 1:
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    with open(out) as fh:
        return fh.read(), r.stdout


def test_bench_two_ranks_equal_one(tmp_path):
    """bench.py's N = 2 flow (weak scaling: 2 x L loci of b37 split by partitionLociUniformly, each
    rank holding the reads overlapping its part, records gathered to rank 0 by sizes + grouped
    send/recv) against one process over the same 2 x L loci with the same two tasks
    (DistributedUtil.scala:584-597, 621-633): identical records."""
    L = "3000000"
    two, out2 = _bench(2, str(tmp_path / "two.json"), ["--length", L])
    one, _ = _bench(1, str(tmp_path / "one.json"), ["--length", L, "--genome-ranks", "2"])
    assert one == two and one.count("], [") > 100
    assert '"n_gpus": 2' in out2


def test_plain_bench_gpus_two_launches_its_ranks():
    """`python bench.py --gpus 2` with no launcher starts two ranks itself (torch.distributed.run,
    before any GPU call) and reports n_gpus 2, with the 2-rank CLI single pass over one BAM of
    the split genome: each rank's region-restricted device ingest, call and gather stages."""
    import json
    env = dict(os.environ, GQ_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--length", "2000000", "--steps", "2", "--warmup", "1",
           "--somatic-length", "0", "--panel-length", "0", "--no-cpu-baseline", "--no-configs3"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2
    sp = line["end_to_end"]["single_pass"]
    assert sp["rc"] == 0 and sp["genotypes"] > 100 and len(sp["per_rank_stages_s"]) == 2
    for rk, st in enumerate(sp["per_rank_stages_s"]):
        assert st["rank"] == rk and st["ingest"] == "device"
        assert st["load_reads"] > 0 and st["call"] > 0 and "gather_s" in st
        assert st["device_ingest"]["plan"] is not None  # region-restricted: planned segments only


def test_rccl_gather_branch_world_one():
    """distributed.gather_germline's RCCL branch (device "cuda:0"): the device-to-device copy of
    the library's result image into a torch tensor and the RCCL collectives, at world size 1 (the
    one-GPU box cannot host two RCCL ranks); records equal the library's own host copy."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_gather_probe.py")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert '"identical": true' in r.stdout


def _synthetic_bam(tmp_path, name, length, depth, seed, index):
    from guacamole_amd import synthetic
    from tests import bam_writer as bw
    p = str(tmp_path / name)
    synthetic.generate(length, depth, seed=synthetic.SEED + seed).write_bam(p)
    if index:
        bw.index_bam(p)
    return p


@pytest.mark.parametrize("index", [False, True])
@pytest.mark.parametrize("parallelism,accuracy", [("5", "0"), ("4", "250")])
def test_germline_two_ranks_device_ingest_equal_one(tmp_path, index, parallelism, accuracy):
    """configs[3]'s multi-GPU ingest on one GPU: each of two ranks decodes on the device only the
    BGZF blocks its tasks need (from the BAI, or by host probes without one) — no rank loads the
    whole file — and the gathered VCF equals one process's.  Each rank holds exactly the reads
    overlapping its tasks' loci (uniform tasks), or those of its micro-partition share when that
    already covers its tasks (by depth: a superset, the same calls)."""
    from guacamole_amd.distributed import ranks_by_position, reads_overlapping
    from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
    from guacamole_amd.reads import InputFilters, load_reads
    bam = _synthetic_bam(tmp_path, "g.bam", 300_000, 30.0, 8, index)
    args = ["germline-threshold", "--reads", bam, "--parallelism", parallelism, "--partition-accuracy", accuracy]
    one = _run(args, 1, str(tmp_path / "one.json"))
    reps = []
    # without an index the probes plan 20 kb back from each range (the default 1 Mb halo would
    # cover this whole 300 kb contig)
    two = _run(args, 2, str(tmp_path / "two.json"), reps, {"GQ_INGEST_HALO": "20000"})
    assert one == two and one.count("\n") > 100
    assert len(reps) == 2
    host = load_reads(bam, InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, has_md_tag=True))
    comp = []
    for rep in sorted(reps, key=lambda r: r["rank"]):
        plan = rep["device_ingest"]["plan"]
        assert rep["ingest"] == "device" and plan is not None and plan["used_index"] == int(index)
        comp.append(plan["comp_bytes"])
    total = os.path.getsize(bam)
    assert sum(comp) < 1.3 * total and max(comp) < 0.75 * total, (comp, total)
    if accuracy == "0":
        loci = LociSet.parse("all").result(host.contig_lengths_map)
        flat = flatten_partitions(partition_loci_uniformly(int(parallelism), loci), host.contig_index())
        rr = ranks_by_position(flat, [0, loci.count // 2, loci.count])
        for rep in reps:
            mine = [np.asarray(a)[rr == rep["rank"]] for a in flat]
            assert rep["reads"] == len(reads_overlapping(host, *mine[:3]))


def test_somatic_two_ranks_device_ingest_equal_one(tmp_path):
    tumor = _synthetic_bam(tmp_path, "t.bam", 200_000, 40.0, 9, True)
    normal = _synthetic_bam(tmp_path, "n.bam", 200_000, 30.0, 10, False)
    args = ["somatic-standard", "--tumor-reads", tumor, "--normal-reads", normal, "--loci", "20:10000-190000",
            "--parallelism", "3", "--partition-accuracy", "0", "--odds", "2"]
    one = _run(args, 1, str(tmp_path / "one.json"))
    reps = []
    two = _run(args, 2, str(tmp_path / "two.json"), reps)
    assert one == two and one.count("\n") > 10
    assert all(r.get("ingest") == "device" for r in reps) and len(reps) == 2


def test_native_context_before_torch_fails_clearly_or_works():
    """The init order of a multi-GPU rank: a native.Context opened before torch
    touches the GPU, then a torch cuda:0 tensor (the gather's device path).  Either it works, or
    check_hip_runtimes names the cause (two HIP runtimes: torch's bundled one and the system's)
    instead of torch's bare "No HIP GPUs are available"."""
    import subprocess
    import sys
    code = ("from guacamole_amd import native\n"
            "ctx = native.Context(0)\n"
            "import torch\n"
            "from guacamole_amd.distributed import check_hip_runtimes, hip_runtimes\n"
            "print('runtimes', hip_runtimes(), flush=True)\n"
            "try:\n"
            "    check_hip_runtimes()\n"
            "except RuntimeError as e:\n"
            "    print('CLEAR', e)\n"
            "    raise SystemExit(3)\n"
            "x = torch.arange(4, device='cuda:0')\n"
            "print('OK', int(x.sum().item()))\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    print(r.stdout, r.stderr[-2000:])
    assert (r.returncode == 0 and "OK 6" in r.stdout) or (r.returncode == 3 and "CLEAR two HIP runtimes" in r.stdout)
    # the supported order: torch first, one runtime, and it works
    code2 = ("import torch\n"
             "torch.cuda.set_device(0)\n"
             "from guacamole_amd import native\n"
             "ctx = native.Context(0)\n"
             "from guacamole_amd.distributed import check_hip_runtimes\n"
             "check_hip_runtimes()\n"
             "print('OK', int(torch.arange(4, device='cuda:0').sum().item()))\n")
    r = subprocess.run([sys.executable, "-c", code2], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0 and "OK 6" in r.stdout, r.stdout + r.stderr[-2000:]
