"""Multi-process data parallelism on the CPU (gloo), mirroring the GPU code paths.

* sync all-reduce and PS-shard (reduce-scatter / all-gather) training of 2 and 4
  replicas equal single-process large-batch training;
* backup workers (replicas_to_aggregate < N) aggregate exactly R replicas/step;
* a localhost ps + worker ClusterSpec job runs the reference-style entrypoint
  (BASELINE config 1) to completion, checkpoints, and resumes.
"""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from mdtf.cluster.launcher import free_port, launch_local_cluster

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _run(world, mode, steps, tmp_path, replicas=None, comm_dtype=None):
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    port = free_port()
    mp.start_processes(dist_helpers.sync_worker, args=(world, port, mode, steps, str(tmp_path), replicas, 4,
                                                       comm_dtype),
                       nprocs=world, join=True, start_method="spawn")
    return [json.load(open(os.path.join(str(tmp_path), "rank%d.json" % r))) for r in range(world)]


@pytest.mark.parametrize("mode", ["allreduce", "sharded"])
@pytest.mark.parametrize("world", [2, 4])
def test_sync_dp_equals_single_process(mode, world, tmp_path):
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    res = _run(world, mode, 5, tmp_path)
    ref = dist_helpers.single_process_reference(world, 5)
    for r in res:
        assert r["step"] == 5
        for name, vals in ref.items():
            assert torch.allclose(torch.tensor(r["weights"][name]), torch.tensor(vals), atol=1e-5), (mode, name)


def test_sharded_gloo_emulation_matches_native_collectives(tmp_path, monkeypatch):
    """on gloo the sharded mode runs its reduce-scatter / all-gather as all-reduces
    (MDTF_GLOO_RS_AR=1, mutating the buckets it is given); the native gloo collectives (=0) must give the same
    weights, and both the single-process large-batch result."""
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("MDTF_GLOO_RS_AR", flag)       # read at import by the spawned ranks
        d = tmp_path / flag
        d.mkdir()
        out[flag] = _run(2, "sharded", 4, d)
    ref = dist_helpers.single_process_reference(2, 4)
    for a, b in zip(out["0"], out["1"]):
        for name in ref:
            ta, tb = torch.tensor(a["weights"][name]), torch.tensor(b["weights"][name])
            assert torch.allclose(ta, tb, atol=1e-6), name
            assert torch.allclose(tb, torch.tensor(ref[name]), atol=1e-5), name


@pytest.mark.parametrize("mode", ["allreduce", "sharded"])
def test_bf16_wire_dtype_matches_fp32_within_tolerance(mode, tmp_path):
    """comm_dtype='bf16': gradients cross the wire in bf16 (half the bytes), masters stay fp32.
    Stated tolerance: after 5 momentum steps every weight is within 2e-2 relative (of the
    largest weight of the tensor) of single-process fp32 training."""
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    res = _run(2, mode, 5, tmp_path, comm_dtype="bf16")
    ref = dist_helpers.single_process_reference(2, 5)
    for r in res:
        for name, vals in ref.items():
            a, b = torch.tensor(r["weights"][name]), torch.tensor(vals)
            assert (a - b).abs().max() <= 2e-2 * b.abs().max() + 1e-4, (mode, name)
    # all replicas agree bit-for-bit (everyone widens the same reduced bf16 values)
    for r in res[1:]:
        for k in res[0]["weights"]:
            assert r["weights"][k] == res[0]["weights"][k]


def test_comm_dtype_resolution(monkeypatch):
    from mdtf.parallel.reducer import resolve_comm_dtype
    from mdtf.config import constants
    assert resolve_comm_dtype() == torch.float32
    assert resolve_comm_dtype("bf16") == torch.bfloat16
    monkeypatch.setenv("MDTF_COMM_DTYPE", "bfloat16")
    assert resolve_comm_dtype() == torch.bfloat16
    with pytest.raises(ValueError):
        resolve_comm_dtype("fp8")
    monkeypatch.setenv("MDTF_BUCKET_MB", "64")
    assert constants.bucket_bytes() == 64 << 20


def test_backup_workers_aggregate_r_of_n(tmp_path):
    res = _run(3, "allreduce", 6, tmp_path, replicas=2)
    assert sum(r["contributed"] for r in res) == 2 * 6          # exactly R contributions per step
    w0 = res[0]["weights"]
    for r in res[1:]:
        for k in w0:
            assert torch.allclose(torch.tensor(r["weights"][k]), torch.tensor(w0[k]), atol=1e-6)


def test_localhost_ps_worker_cluster_and_resume(tmp_path):
    md = str(tmp_path / "model")
    script = os.path.join(ROOT, "distribute.py")
    codes = launch_local_cluster([script, "--model_dir=%s" % md, "--epochs=1"], num_ps=1, num_workers=1,
                                 timeout_s=900)
    assert codes == [0, 0]
    from mdtf.train.saver import latest_checkpoint
    ck = latest_checkpoint(md)
    assert ck and ck.endswith("model.ckpt-100")
    # resume: epochs=2 -> continues from step 100 to 200
    codes = launch_local_cluster([script, "--model_dir=%s" % md, "--epochs=2"], num_ps=1, num_workers=1,
                                 timeout_s=900)
    assert codes == [0, 0]
    assert latest_checkpoint(md).endswith("model.ckpt-200")
    from mdtf.ckpt.tensor_bundle import BundleReader
    r = BundleReader(latest_checkpoint(md))
    assert int(r.get_tensor("global_step")) == 200
    assert "conv1/weights" in r and "conv1/weights/Adam" in r and "beta1_power" in r


def test_two_workers_one_ps_sharded(tmp_path):
    md = str(tmp_path / "model2")
    script = os.path.join(ROOT, "distribute.py")
    codes = launch_local_cluster([script, "--model_dir=%s" % md, "--epochs=1"], num_ps=1, num_workers=2,
                                 timeout_s=900)
    assert codes == [0, 0, 0]


def test_eval_mode_restores_checkpoint(tmp_path):
    md = str(tmp_path / "model3")
    script = os.path.join(ROOT, "distribute.py")
    assert launch_local_cluster([script, "--model_dir=%s" % md, "--epochs=1"], 1, 1, timeout_s=900) == [0, 0]
    port = free_port()
    out = subprocess.run([sys.executable, script, "--job_name=worker", "--task_index=0", "--mode=Eval",
                          "--worker_hosts=127.0.0.1:%d" % port, "--ps_hosts=none", "--model_dir=%s" % md],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-3000:]
    assert "Eval: {" in out.stdout and "model.ckpt-100" in out.stdout


def test_async_ps_two_ps_two_workers(tmp_path):
    """Async PS mode: variables sharded over 2 PS ranks, 2 workers push/pull independently."""
    md = str(tmp_path / "async")
    script = os.path.join(ROOT, "distribute.py")
    codes = launch_local_cluster([script, "--model_dir=%s" % md, "--ps_mode=async"], num_ps=2, num_workers=2,
                                 timeout_s=900)
    assert codes == [0, 0, 0, 0]
    from mdtf.ckpt.tensor_bundle import BundleReader
    from mdtf.train.saver import latest_checkpoint
    ck = latest_checkpoint(md)
    r = BundleReader(ck)
    assert r.num_shards == 2
    shards = {r.entries[k].shard_id for k in r.keys()}
    assert shards == {0, 1}                     # variables live on both PS tasks
    assert int(r.get_tensor("global_step")) >= 100


def test_sync_ps_backup_workers_do_not_wait_for_a_straggler(tmp_path):
    """ps_mode=sync_ps, 3 workers, replicas_to_aggregate=2 (distribute_train.py:146-160): each PS version is the
    mean of the first 2 pushes computed on it; worker 2 sleeps 4x its own forward/backward time per step (5x
    slower whatever the host's load), so its pushes are mostly late and dropped, and the two fast workers reach the
    last step without waiting for it (latency hiding)."""
    md = str(tmp_path / "syncps")
    out = str(tmp_path / "stats")
    os.makedirs(out)
    script = os.path.join(ROOT, "distribute.py")
    codes = launch_local_cluster([script, "--model_dir=%s" % md, "--ps_mode=sync_ps", "--replicas_to_aggregate=2"],
                                 num_ps=1, num_workers=3, timeout_s=900,
                                 extra_env={"MDTF_STRAGGLER": "worker:2:x4", "MDTF_BENCH_OUT": out})
    assert codes == [0, 0, 0, 0]
    ps = json.load(open(os.path.join(out, "ps0.json")))
    assert ps["mode"] == "sync_ps R=2" and ps["batched_max"] == 2
    assert ps["updates"] == 100                 # one update per global step, each the mean of exactly 2 pushes
    assert ps["dropped"] >= 10, ps              # the straggler's late pushes were discarded, not waited for
    w = [json.load(open(os.path.join(out, "worker%d.json" % i))) for i in range(3)]
    assert w[2]["steps_done"] < min(w[0]["steps_done"], w[1]["steps_done"]), w
    from mdtf.train.saver import latest_checkpoint
    from mdtf.ckpt.tensor_bundle import BundleReader
    assert int(BundleReader(latest_checkpoint(md)).get_tensor("global_step")) == 100


@pytest.mark.slow
def test_fault_injection_restart_resumes_from_checkpoint(tmp_path):
    """Kill worker 1 at global step 37; the heartbeat watchdog stops the surviving tasks, the supervisor
    restarts the job, the chief resumes from the last checkpoint (step 30) and training completes."""
    md = str(tmp_path / "ft")
    script = os.path.join(ROOT, "distribute.py")
    env = {"MDTF_FAULT_STEP": "37", "MDTF_FAULT_TASK": "worker:1", "MDTF_HEARTBEAT_INTERVAL": "0.5",
           "MDTF_HEARTBEAT_TIMEOUT": "5"}
    codes = launch_local_cluster([script, "--model_dir=%s" % md, "--epochs=1", "--save_checkpoint_steps=10"],
                                 num_ps=1, num_workers=2, extra_env=env, timeout_s=600, max_restarts=2,
                                 log_dir=str(tmp_path / "logs"))
    assert codes == [0, 0, 0]
    assert launch_local_cluster.last_attempts == 1
    from mdtf.train.saver import latest_checkpoint
    from mdtf.ckpt.tensor_bundle import BundleReader
    ck = latest_checkpoint(md)
    assert ck.endswith("model.ckpt-100")
    assert int(BundleReader(ck).get_tensor("global_step")) == 100
    logs = tmp_path / "logs"
    assert "injected fault at global step 37" in (logs / "task2.attempt0.log").read_text()
    resumed = (logs / "task1.attempt1.log").read_text()
    assert "Restored from checkpoint" in resumed and "model.ckpt-30 (global_step 30)" in resumed


def test_heartbeat_detects_silent_peer():
    """Two heartbeats on one TCPStore: when one stops beating (without 'done'), the other reports it."""
    import torch.distributed as dist
    from mdtf.cluster.health import Heartbeat
    port = free_port()
    store = dist.TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False)
    failed = []
    a = Heartbeat(store, 0, 2, interval=0.1, timeout=0.6, on_failure=failed.append).start()
    b = Heartbeat(store, 1, 2, interval=0.1, timeout=0.6, on_failure=failed.append).start()
    import time
    time.sleep(0.5)
    assert failed == []
    b.stop(done=False)            # rank 1 goes silent
    t0 = time.time()
    while not failed and time.time() - t0 < 5:
        time.sleep(0.05)
    a.stop()
    assert failed == [1]
    # a peer that finishes cleanly is never reported
    failed.clear()
    c = Heartbeat(store, 0, 2, interval=0.1, timeout=0.4, prefix="mdtf/hb2", on_failure=failed.append).start()
    d = Heartbeat(store, 1, 2, interval=0.1, timeout=0.4, prefix="mdtf/hb2", on_failure=failed.append).start()
    time.sleep(0.3)
    d.stop(done=True)
    time.sleep(1.0)
    c.stop()
    assert failed == []


@pytest.mark.parametrize("save_steps", [None, 2])
def test_sharded_collective_checkpoint_through_monitored_session(save_steps, tmp_path):
    """Saving in sharded mode all-gathers the optimizer shards; the default chief-only, 600 s
    hook would hang the chief at the first save.  Every replica now saves on the same steps."""
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    from mdtf.train.saver import latest_checkpoint
    from mdtf.ckpt.tensor_bundle import BundleReader
    port = free_port()
    ctx = mp.start_processes(dist_helpers.sharded_ckpt_worker, args=(2, port, 5, str(tmp_path), save_steps),
                             nprocs=2, join=False, start_method="spawn")
    import time
    deadline = time.time() + 180
    while not ctx.join(timeout=5):
        if time.time() > deadline:
            for p in ctx.processes:
                p.kill()
            pytest.fail("sharded replicas hung in the collective checkpoint save")
    ck = latest_checkpoint(str(tmp_path / "model"))
    assert ck and ck.endswith("model.ckpt-5")
    r = BundleReader(ck)
    assert "dense/w/Adam" in r and int(r.get_tensor("global_step").item()) == 5
    if save_steps == 2:
        import glob
        assert os.path.exists(str(tmp_path / "model" / "model.ckpt-4.index"))


def test_restore_when_checkpoint_visible_only_on_chief(tmp_path):
    """a node-local model_dir.  The chief reads the bundle and broadcasts it; every
    replica (sharded mode: its own Adam shard) resumes from the same state."""
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    from mdtf.ckpt.tensor_bundle import BundleReader
    from mdtf.train.saver import latest_checkpoint
    mp.start_processes(dist_helpers.sharded_ckpt_worker, args=(2, free_port(), 3, str(tmp_path), None),
                       nprocs=2, join=True, start_method="spawn")
    ck = latest_checkpoint(str(tmp_path / "model"))
    assert ck and ck.endswith("model.ckpt-3")
    mp.start_processes(dist_helpers.hidden_ckpt_restore_worker, args=(2, free_port(), str(tmp_path)),
                       nprocs=2, join=True, start_method="spawn")
    res = [json.load(open(str(tmp_path / ("resume%d.json" % r)))) for r in range(2)]
    r = BundleReader(ck)
    for rec in res:
        assert rec["step"] == 3 and rec["restored"] == ck
        for name, vals in rec["weights"].items():
            assert torch.allclose(torch.tensor(vals), r.get_tensor(name).float().reshape(torch.tensor(vals).shape))
    assert res[0]["adam_m"] == res[1]["adam_m"]
    assert any(abs(x) > 0 for x in res[0]["adam_m"])


@pytest.mark.parametrize("agree", ["sync", "async"])
def test_coordinated_recovery_one_replica_aborts(tmp_path, agree):
    """ONE of two sync replicas raises AbortedError after step 5 (reference distribute_train.py:169-180: the
    recoverable MonitoredTrainingSession).  Both replicas agree on the recovery at a step boundary (sync: the
    next one; async: the code posted at the next boundary is read one boundary later), re-create their sessions
    in process from the chief's latest checkpoint, and finish at the same global step with the weights of an
    uninterrupted run."""
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    res = {}
    for tag, fault in (("ref", None), ("run", 5)):
        d = tmp_path / tag
        d.mkdir()
        mp.start_processes(dist_helpers.recovery_worker, args=(2, free_port(), 8, str(d), fault, "worker:1", "abort",
                                                               agree),
                           nprocs=2, join=True, start_method="spawn")
        res[tag] = [json.load(open(str(d / ("rank%d.json" % r)))) for r in range(2)]
    ref, run = res["ref"], res["run"]
    assert [r["step"] for r in run] == [8, 8] and [r["recoveries"] for r in run] == [1, 1]
    assert [r["recoveries"] for r in ref] == [0, 0]
    assert run[0]["runs"] == run[1]["runs"]
    if agree == "sync":
        assert run[0]["runs"] == ref[0]["runs"] + 1     # step 5 re-runs from the step-4 state
    for k, w in ref[0]["weights"].items():
        for r in run:
            assert torch.allclose(torch.tensor(r["weights"][k]), torch.tensor(w), atol=1e-6), k


def test_coordinated_recovery_error_inside_the_step(tmp_path):
    """ONE of two sync replicas raises AbortedError from INSIDE its train op (after the step's collectives and
    update: ``FaultInjectionHook`` mode ``abort_in_step``), not from a hook.  The failing replica holds the
    error, both replicas agree at the next step boundary, restore the chief's step-4 checkpoint in process and
    finish at the same global step with the weights of an uninterrupted run (reference
    distribute_train.py:169-180)."""
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    res = {}
    for tag, fault in (("ref", None), ("run", 5)):
        d = tmp_path / tag
        d.mkdir()
        mp.start_processes(dist_helpers.recovery_worker, args=(2, free_port(), 8, str(d), fault, "worker:1",
                                                               "abort_in_step"),
                           nprocs=2, join=True, start_method="spawn")
        res[tag] = [json.load(open(str(d / ("rank%d.json" % r)))) for r in range(2)]
    ref, run = res["ref"], res["run"]
    assert [r["step"] for r in run] == [8, 8] and [r["recoveries"] for r in run] == [1, 1]
    assert [r["agreements"] for r in run] == [run[0]["agreements"]] * 2       # lockstep boundaries
    # the failing replica retried its run inside the same call, so its peer made one call more
    assert run[1]["runs"] == run[0]["runs"] - 1
    for k, w in ref[0]["weights"].items():
        for r in run:
            assert torch.allclose(torch.tensor(r["weights"][k]), torch.tensor(w), atol=1e-6), k


def test_coordinated_recovery_hook_error_in_before_run_async(tmp_path):
    """ONE of two replicas' hooks raises a RECOVERABLE AbortedError from before_run under the async agreement
    (``MDTF_AGREE=async``).  The step it posted the code with still runs on both replicas (no run context, so its
    after_run hooks are skipped), every replica reads RECOVER at the next boundary, restores the chief's
    checkpoint in process and finishes at the same global step with the weights of an uninterrupted run
    (reference distribute_train.py:169-180)."""
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    res = {}
    for tag, fault in (("ref", None), ("run", 5)):
        d = tmp_path / tag
        d.mkdir()
        mp.start_processes(dist_helpers.recovery_worker, args=(2, free_port(), 8, str(d), fault, "worker:1",
                                                               "abort_before_run", "async"),
                           nprocs=2, join=True, start_method="spawn")
        res[tag] = [json.load(open(str(d / ("rank%d.json" % r)))) for r in range(2)]
    ref, run = res["ref"], res["run"]
    assert [r["step"] for r in run] == [8, 8] and [r["recoveries"] for r in run] == [1, 1]
    assert [r["agreements"] for r in run] == [run[0]["agreements"]] * 2
    for k, w in ref[0]["weights"].items():
        for r in run:
            assert torch.allclose(torch.tensor(r["weights"][k]), torch.tensor(w), atol=1e-6), k


def test_fatal_hook_error_stops_every_replica(tmp_path):
    """A non-recoverable error in one replica's before_run still joins the step-boundary agreement: the peer
    stops at that boundary with an error instead of waiting in the next step's collectives."""
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    d = tmp_path / "fatal"
    d.mkdir()
    mp.start_processes(dist_helpers.fatal_hook_worker, args=(2, free_port(), str(d)), nprocs=2, join=True,
                       start_method="spawn")
    out = [json.load(open(str(d / ("rank%d.json" % r)))) for r in range(2)]
    assert out[1]["error"].startswith("ValueError") and "bug in a hook" in out[1]["error"]
    assert out[0]["error"].startswith("RuntimeError") and "non-recoverable" in out[0]["error"]
    assert out[0]["step"] == out[1]["step"] == 4        # async agreement: the posted step still ran everywhere


@pytest.mark.parametrize("fake", [False, True])
def test_backup_device_path_only_on_one_host(tmp_path, fake):
    """The device-clock backup-worker path (clocks calibrated against one host's monotonic clock) is taken only
    when every rank of the group is on one host; that is decided from the ranks' host names, not from torchrun's
    env, which the ClusterSpec launcher does not set (reference distribute.py:37-38: workers on several hosts)."""
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    mp.start_processes(dist_helpers.host_check_worker, args=(2, free_port(), str(tmp_path), fake), nprocs=2,
                       join=True, start_method="spawn")
    out = [json.load(open(str(tmp_path / ("host%d.json" % r))))["single"] for r in range(2)]
    assert out == [not fake, not fake]
