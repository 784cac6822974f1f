"""The driver's multi-GPU launch of bench.py, rehearsed on the CPU.

The round-end driver runs ``python -m torch.distributed.run --nnodes=1 --nproc-per-node N
--master-addr 127.0.0.1 --master-port P bench.py --gpus N ...`` (one rank per GPU over RCCL).
The same command with 2 ranks on gloo (no GPU here) walks the whole path: Server.from_env, the
bucketed gradient reduction in both sync modes, the MAX-over-ranks timing and rank 0's JSON line.
Tiny images keep ResNet-50 cheap on the CPU.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.slow
@pytest.mark.parametrize("mode", ["allreduce", "sharded"])
def test_bench_torchrun_two_ranks(mode):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--batch", "2", "--image_size", "32", "--mode", mode]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("MDTF_HIP_GRAPH", None)
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]          # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["global_batch"] == 4 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["grad_sync"] == mode
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    assert rec["loss_last"] == rec["loss_last"]           # finite
    assert rec["comm"] == {"backend": "gloo", "ranks_in_collective": 2}


def _one_json(out):
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]          # rank 0 only
    return json.loads(lines[0])


@pytest.mark.slow
@pytest.mark.parametrize("mode", ["allreduce", "sharded"])
def test_bench_gpus_flag_self_launches_eight_ranks(mode):
    """``python bench.py --gpus 8`` without torchrun spawns 8 ranks (here gloo on the CPU) and
    reports them; it used to ignore --gpus and time one process."""
    cmd = [sys.executable, "bench.py", "--gpus", "8", "--steps", "2", "--warmup", "1", "--batch", "1",
           "--image_size", "32", "--mode", mode]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("MDTF_HIP_GRAPH", None)
    rec = _one_json(subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1200))
    assert rec["n_gpus"] == 8 and rec["config"]["parallelism"] == "dp8"
    assert rec["config"]["global_batch"] == 8 and rec["config"]["grad_sync"] == mode
    assert rec["per_gpu_images_per_sec"] == pytest.approx(rec["value"] / 8, abs=0.01)


@pytest.mark.slow
def test_bench_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "4"], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode != 0 and "launch mismatch" in out.stderr


@pytest.mark.slow
def test_bert_bench_eight_ranks_cpu():
    cmd = [sys.executable, "bench/bert_bench.py", "--gpus", "8", "--size", "tiny", "--batch", "2", "--seq", "32",
           "--steps", "2", "--warmup", "1", "--mode", "sharded"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    rec = _one_json(subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900))
    assert rec["n_gpus"] == 8 and rec["config"]["global_batch"] == 16 and rec["impl"] == "mdtf"
    assert rec["config"]["grad_sync"] == "sharded" and rec["value"] > 0


@pytest.mark.slow
def test_collectives_sweep_runs_on_gloo():
    """bench/collectives.py (the bucket-size sweep for an 8-GPU node) runs end to end on 4 gloo ranks."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench/collectives.py",
           "--sizes_mb", "1,2", "--iters", "2", "--warmup", "1"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    recs = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(recs) >= 2 * 2 * 3            # 2 dtypes x 2 sizes x 3 collectives
    assert all(r["busbw_GBps"] > 0 for r in recs)


@pytest.mark.slow
def test_bench_bf16_wire_two_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--batch", "2", "--image_size", "32", "--comm_dtype", "bf16",
           "--bucket_mb", "8"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["config"]["comm_dtype"] == "bf16"


@pytest.mark.slow
def test_async_ps_bench_two_ps_six_workers_cpu():
    """BASELINE config 5's topology (2 ps + 6 workers, one process each) on gloo: every worker reports its
    throughput, every PS its staleness and busy/idle split; the data plane never waits on the store."""
    cmd = [sys.executable, "bench/async_ps_bench.py", "--cpu", "--num_ps", "2", "--num_workers", "6", "--depth", "50",
           "--image", "32", "--batch", "2", "--steps", "2", "--warmup", "1", "--timeout_s", "500"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=560)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-2000:])
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert len(rec["per_worker"]) == 6 and all(r > 0 for r in rec["per_worker"])
    assert len(rec["ps"]) == 2
    for ps in rec["ps"]:
        # the gloo run polls the same posted-receive service loop RCCL runs (helper-thread completion flags),
        # applies every completed payload in one fused pass, and never calls the store while serving
        assert ps["updates"] >= 18 and ps["poll"] == "threaded-gloo" and ps["store_calls"] == 0
        assert 1 <= ps["applies"] <= ps["updates"] and ps["batched_max"] >= 1
        assert ps["mean_staleness"] >= 1.0          # 6 workers + the worker-side push/compute overlap


@pytest.mark.slow
def test_async_ps_single_worker_staleness_counts_the_overlap():
    """One worker: its push of step t travels while forward/backward of step t+1 runs on the weights it already
    holds, so every gradient after the first is computed one PS version behind (the push header
    must carry the version the gradient was computed on, not the reply that arrived meanwhile)."""
    cmd = [sys.executable, "bench/async_ps_bench.py", "--cpu", "--num_ps", "1", "--num_workers", "1", "--depth", "50",
           "--image", "32", "--batch", "2", "--steps", "6", "--warmup", "1", "--timeout_s", "300"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=360)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-2000:])
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    ps = rec["ps"][0]
    assert ps["max_staleness"] == 1 and ps["mean_staleness"] >= 0.8, ps


@pytest.mark.slow
def test_async_ps_bert_padded_decoder_cpu():
    """BERT's tied decoder reserves zero pad rows after the word embedding and the MLM bias in
    the flat buffers; the PS must rebuild the same flat layout from the variable spec, or the chief's initial
    send and every push / pull mismatch in size (a gloo size error, an RCCL hang).  2 ps + 2 workers, BERT-tiny."""
    cmd = [sys.executable, "bench/async_ps_bench.py", "--cpu", "--model", "bert", "--num_ps", "2", "--num_workers", "2",
           "--seq", "32", "--batch", "2", "--steps", "2", "--warmup", "1", "--timeout_s", "300"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=360)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-2000:])
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["unit"] == "sequences/sec" and len(rec["per_worker"]) == 2 and all(r > 0 for r in rec["per_worker"])
    assert all(ps["updates"] >= 6 for ps in rec["ps"])
