"""The multi-GPU product path (configs[3] shape) on one GPU: the CLI launched by
torch.distributed.run with two ranks (gloo gather, both ranks on cuda:0) writes exactly what the
single-process run with the same task partition writes.  Cuts between the ranks fall inside
chrM's 150x coverage, so reads straddling them go to both ranks (DistributedUtil.scala:584-597)."""
import os
import socket
import subprocess
import sys

import pytest

from conftest import fixture

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, world, out):
    env = dict(os.environ, GQ_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    if world == 1:
        cmd = [sys.executable, "-m", "guacamole_amd"] + args + ["--out", out]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "guacamole_amd"] + args + ["--out", out]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
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
            "--no-single-pass",
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


def test_rccl_gather_branch_world_one():
    """distributed.gather_germline's RCCL branch (device "cuda:0"): the device-to-device copy of
    the library's result image into a torch tensor and the RCCL collectives, at world size 1 (the
    one-GPU box cannot host two RCCL ranks); records equal the library's own host copy."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_gather_probe.py")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert '"identical": true' in r.stdout
