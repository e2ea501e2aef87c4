"""bench.py on the GPU, run as the driver runs it (a child process): the C3 job
at full size through the strong-scaling path (JobPlan + JobGather) with every
count and location checked against the oracle; several ranks rehearsed on one
GPU over gloo; RCCL oversubscription refused."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(args, env_extra=None, timeout=900, torchrun=0):
    """bench.py as a child process; torchrun=N: under `python -m
    torch.distributed.run --nproc-per-node N` (the driver's multi-GPU launch)."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "FMX_BENCH_BACKEND", "FMX_BENCH_DIST"):
        env.pop(k, None)
    env.update(env_extra or {})
    launcher = [sys.executable, "-u"]
    if torchrun:
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        launcher += ["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={torchrun}",
                     "--master-addr=127.0.0.1", f"--master-port={port}"]
    p = subprocess.run(launcher + [os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                       text=True, timeout=timeout, env=env)
    sys.stderr.write(p.stderr[-4000:])
    return p


def last_json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


def test_c3_full_job_one_gpu():
    """BASELINE configs[2] (10 M x 20 bp over 1 Gbp) on one GPU: the job is
    planned (256 batches of ~39 k, one grouped launch of 256), every launch's
    results are written into the exactly sized gather slabs, the job's flat
    (offsets, locations) is assembled on the device, and rank 0 compares all
    10 M counts and every location with the CPU oracle."""
    p = run_bench(["--config", "c3", "--verify-job", "--no-cpu", "--no-blob-layout", "--min-seconds", "0.05",
                   "--warmup", "0"])
    assert p.returncode == 0, p.stderr[-3000:]
    r = last_json(p.stdout)
    assert r["scaling"] == "strong" and r["config"]["global_batch"] == 10_000_000
    assert r["parity"]["scope"] == "every pattern of the job" and r["parity"]["patterns"] == 10_000_000
    assert r["parity"]["bit_exact_vs_cpu"], r["parity"]
    g = r["gather"]
    assert g["assembly_ok"] and g["needs_stable"] and g["assembled_patterns"] == 10_000_000
    assert g["plan"]["batches_per_rank"] % 128 == 0 and g["plan"]["launch_groups"] == 1
    assert r["config"]["launch_order"].startswith("grouped")
    assert r["self_location_check"] and r["n_gpus"] == 1 and r["ranks"] == 1


def test_rccl_world1_strong_job():
    """The RCCL path on the one GPU of the box: bench.py
    under torchrun --nproc-per-node 1 with the nccl backend and the process
    group up for one rank (FMX_BENCH_DIST=1) — the blob self-broadcast and
    checksum (replicate_blob), every launch group's results all-gathered by
    RCCL inside the timed step (JobGather.gather), the job assembled from the
    gathered slabs (assemble) and all 800,000 patterns checked against the
    oracle (--verify-job).  So the driver's 8-GPU run is not this code's first
    contact with RCCL."""
    p = run_bench(["--config", "c3", "--text-len", "50000000", "--total-patterns", "800000", "--verify-job",
                   "--no-cpu", "--min-seconds", "0.05", "--warmup", "0"],
                  env_extra={"FMX_BENCH_DIST": "1"}, torchrun=1)
    assert p.returncode == 0, p.stderr[-3000:]
    r = last_json(p.stdout)
    assert r["backend"] == "nccl" and r["rccl_world_size"] == 1 and r["ranks"] == 1
    g = r["gather"]
    assert g["inside_timed_step"] and g["collectives_per_launch"] == 1 and g["assembly_ok"]
    assert g["gathered_over_result"] <= 1.0 + 1e-9
    rep = r["blob_replication"]
    assert rep["identical"] and rep["bytes"] > 0 and "broadcast" in rep["how"]
    assert r["parity"]["bit_exact_vs_cpu"] and r["parity"]["patterns"] == 800_000
    assert r["hbm_per_rank"]["gather_slabs"] > 0
    # one launch group per stream (--strong-groups default), each of 256 / 2 batches
    assert g["plan"]["launch_groups"] == r["config"]["streams"] == 2
    assert r["config"]["batches_per_launch"] == 128 and g["plan"]["batches_per_rank"] == 256


@pytest.mark.parametrize("policy", ["all", "counts"])
def test_rccl_world1_weak_gather(policy):
    """c2-shaped weak scaling under torchrun with one RCCL rank: each launch
    group's counts and locations (`--gather all`) or counts alone (`--gather
    counts`: the locations gathered once after the timed region) all-gathered
    by RCCL inside the timed step; the assembled results hold this rank's part
    intact, and the line states what each policy moves and needs."""
    p = run_bench(["--config", "c2", "--text-len", "20000000", "--patterns", "20000", "--group", "64", "--steps",
                   "16", "--batches", "16", "--no-cpu", "--min-seconds", "0.05", "--warmup", "0",
                   "--gather", policy], env_extra={"FMX_BENCH_DIST": "1"}, torchrun=1)
    assert p.returncode == 0, p.stderr[-3000:]
    r = last_json(p.stdout)
    assert r["backend"] == "nccl" and r["rccl_world_size"] == 1 and r["scaling"] == "weak"
    g = r["gather"]
    assert g["inside_timed_step"] and g["collectives_per_launch"] == 1 and g["assembly_ok"]
    assert g["assembled_patterns"] == r["config"]["distinct_batches"] * 20000
    assert g["policy"] == policy and g["bytes_gathered_per_pass"] == g["bytes_per_pass"][policy]
    assert g["bytes_per_pass"]["counts"] < g["bytes_per_pass"]["all"]
    assert g["required_gbs_per_gpu_at_n8"]["all"] > g["required_gbs_per_gpu_at_n8"]["counts"] > 0


def test_rccl_oversubscription_refused():
    """Two RCCL ranks on a one-GPU box: refused before any GPU work."""
    import torch
    n = torch.cuda.device_count() + 1
    p = run_bench(["--gpus", str(n)], timeout=300)
    assert p.returncode == 2 and "refusing to oversubscribe" in p.stderr


def test_gloo_two_ranks_one_gpu_strong():
    """FMX_BENCH_BACKEND=gloo bench.py --gpus 2: bench.py starts both ranks
    itself; they share cuda:0 and the line says so (n_gpus 1, ranks 2, no RCCL
    world).  A sharded job with the in-step gathers (one collective per launch
    group); the assembled job equals the oracle's answer."""
    p = run_bench(["--gpus", "2", "--config", "c3", "--text-len", "50000000", "--total-patterns", "800000",
                   "--verify-job", "--no-cpu", "--min-seconds", "0.05", "--warmup", "0"],
                  env_extra={"FMX_BENCH_BACKEND": "gloo"})
    assert p.returncode == 0, p.stderr[-3000:]
    r = last_json(p.stdout)
    assert r["n_gpus"] == 1 and r["ranks"] == 2 and r["rccl_world_size"] is None and r["backend"] == "gloo"
    g = r["gather"]
    assert g["inside_timed_step"] and g["collectives_per_launch"] == 1 and g["assembly_ok"]
    assert g["gathered_over_result"] <= 1.25
    assert g["plan"]["patterns_per_rank"] == [400_000, 400_000]
    # with gathers: one launch group per stream and rank (each group's gather overlaps the other's search)
    assert g["plan"]["launch_groups"] == r["config"]["streams"] == 2 and r["config"]["batches_per_launch"] == 128
    assert r["parity"]["bit_exact_vs_cpu"] and r["parity"]["patterns"] == 800_000
    rep = r["blob_replication"]  # rank 0's blob broadcast to rank 1, checksums equal
    assert rep["identical"] and rep["bytes"] > 0


def test_gloo_two_ranks_weak_gather():
    """c2-style weak scaling on two ranks (gloo, one GPU): every launch
    group's results are all-gathered inside the timed step (one collective
    per launch, exactly sized slabs), the job assembled on the device holds
    this rank's part intact, and the padding stays under 1.25x."""
    p = run_bench(["--gpus", "2", "--config", "c2", "--text-len", "20000000", "--patterns", "20000", "--group", "64",
                   "--steps", "16", "--batches", "16", "--no-cpu", "--min-seconds", "0.05", "--warmup", "0"],
                  env_extra={"FMX_BENCH_BACKEND": "gloo"})
    assert p.returncode == 0, p.stderr[-3000:]
    r = last_json(p.stdout)
    assert r["ranks"] == 2 and r["n_gpus"] == 1 and r["scaling"] == "weak"
    g = r["gather"]
    assert g["inside_timed_step"] and g["collectives_per_launch"] == 1 and g["assembly_ok"]
    assert g["bytes_gathered_per_pass"] <= 1.25 * g["result_bytes_per_pass"]
    assert g["assembled_patterns"] == 2 * r["config"]["distinct_batches"] * 20000
    assert 0 < r["value"] <= g["value_compute_only"] * 1.5
