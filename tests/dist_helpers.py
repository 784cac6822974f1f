"""Worker bodies for the multi-process (gloo, CPU) tests; imported by spawned processes."""
import json
import os

import torch


def _teardown(server):
    """End a spawned rank after its results are written.  Server.from_env leaves the process group to its launcher
    (torchrun); these ranks have none.  Tearing the gloo group and its TCPStore down through destructors still
    aborted a rank now and then on a loaded 8-CPU machine ("terminate called without an active exception", ~1 run
    in 3 of the suite under -n 8) after the test's work was done, so: stop the heartbeat, meet every rank at a
    barrier (the store host stays up until all ranks are past it), and leave without running destructors."""
    import sys
    import torch.distributed as dist
    if getattr(server, "heartbeat", None) is not None:
        server.heartbeat.stop(done=True)
    code = 0
    if dist.is_initialized():
        try:
            dist.barrier()
        except Exception as e:  # noqa: BLE001 - a peer that crashed or hung in shutdown must fail the test
            sys.stderr.write("teardown barrier failed: %r\n" % (e,))
            code = 1
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)


def _linear_setup(rank, world, batch, seed=0):
    import mdtf
    from mdtf.runtime import Loss, Model, Net, Tower
    from mdtf.train import variables as V

    class Lin(Model):
        def inference(self, x):
            w = V.get_variable("dense/w", [8, 3], initializer=V.constant_initializer(0.1))
            b = V.get_variable("dense/b", [3], initializer=V.constant_initializer(0.0))
            h = V.get_variable("dense2/w", [3, 1], initializer=V.constant_initializer(0.2))
            return torch.tanh(x @ w + b) @ h

    class MSE(Loss):
        def loss(self, p, t):
            return ((p - t) ** 2).mean()

    g = torch.Generator().manual_seed(seed)
    xs = torch.randn(world * batch, 8, generator=g)
    ys = torch.randn(world * batch, 1, generator=g)
    x_ph = mdtf.placeholder(torch.float32, [None, 8])
    y_ph = mdtf.placeholder(torch.float32, [None, 1])
    return Lin, MSE, xs, ys, x_ph, y_ph, Tower, Net


def sync_worker(rank, world, port, mode, steps, out_dir, replicas=None, batch=4, comm_dtype=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import mdtf
    from mdtf.cluster import Server
    from mdtf.train import variables as V
    server = Server.from_env(backend="gloo")
    Lin, MSE, xs, ys, x_ph, y_ph, Tower, Net = _linear_setup(rank, world, batch)
    base = mdtf.train.MomentumOptimizer(0.1, 0.9)
    tg = []
    tower = Tower(Net(Lin()), "tower_0/", tg, x_ph, y_ph, MSE(), base, batch_size=batch)
    _, loss, _ = tower.process()
    opt = mdtf.train.SyncReplicasOptimizer(base, replicas_to_aggregate=replicas or world, total_num_replicas=world,
                                           mode=mode, bucket_bytes=64,     # tiny buckets: several per group
                                           comm_dtype=comm_dtype)
    gs = mdtf.train.get_or_create_global_step()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)
    hook = opt.make_session_run_hook(rank == 0)
    sess = mdtf.train.MonitoredTrainingSession(is_chief=rank == 0, hooks=[hook], log_step_count_steps=0,
                                               server=server)
    lo, hi = rank * batch, (rank + 1) * batch
    contributed = 0
    for _ in range(steps):
        sess.run(op, feed_dict={x_ph: xs[lo:hi], y_ph: ys[lo:hi]})
        contributed += int(op.last_contributed)
    sess.close()
    op.reducer.gather_full_master()
    w = {v.name: v.master.tolist() for v in V.get_store().trainable_variables()}
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump({"weights": w, "contributed": contributed, "step": gs.value()}, f)
    _teardown(server)


def single_process_reference(world, steps, batch=4):
    import mdtf
    from mdtf.train import step as S
    from mdtf.train import variables as V
    V.reset_default_graph()
    S.reset()
    Lin, MSE, xs, ys, x_ph, y_ph, Tower, Net = _linear_setup(0, world, batch)
    opt = mdtf.train.MomentumOptimizer(0.1, 0.9)
    tg = []
    tower = Tower(Net(Lin()), "tower_0/", tg, x_ph, y_ph, MSE(), opt, batch_size=world * batch)
    tower.process()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    for _ in range(steps):
        sess.run(op, feed_dict={x_ph: xs, y_ph: ys})
    return {v.name: v.master.tolist() for v in V.get_store().trainable_variables()}


def sharded_ckpt_worker(rank, world, port, steps, out_dir, save_steps=None):
    """Sharded-mode replicas with the factory's default (time-triggered) checkpoint settings:
    the collective save must run on every replica at the same steps (session.py)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import mdtf
    from mdtf.cluster import Server
    from mdtf.train import hooks as H
    server = Server.from_env(backend="gloo")
    batch = 4
    Lin, MSE, xs, ys, x_ph, y_ph, Tower, Net = _linear_setup(rank, world, batch)
    base = mdtf.train.AdamOptimizer(0.01)
    tg = []
    tower = Tower(Net(Lin()), "tower_0/", tg, x_ph, y_ph, MSE(), base, batch_size=batch)
    tower.process()
    opt = mdtf.train.SyncReplicasOptimizer(base, replicas_to_aggregate=world, total_num_replicas=world,
                                           mode="sharded")
    gs = mdtf.train.get_or_create_global_step()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)
    md = os.path.join(out_dir, "model")
    kw = {} if save_steps is None else dict(save_checkpoint_steps=save_steps)
    lo, hi = rank * batch, (rank + 1) * batch
    with mdtf.train.MonitoredTrainingSession(is_chief=rank == 0, checkpoint_dir=md, log_step_count_steps=0,
                                             hooks=[H.StopAtStepHook(last_step=steps)], server=server,
                                             **kw) as sess:
        while not sess.should_stop():
            sess.run(op, feed_dict={x_ph: xs[lo:hi], y_ph: ys[lo:hi]})
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump({"step": gs.value()}, f)
    _teardown(server)


def hidden_ckpt_restore_worker(rank, world, port, out_dir):
    """Resume in sharded mode where only the chief can see model_dir (node-local disk): rank 1's
    os.path.exists is blinded to the checkpoint files, so the chief must read and broadcast them."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    md = os.path.join(out_dir, "model")
    if rank != 0:
        real = os.path.exists
        os.path.exists = lambda p: False if str(p).startswith(md) else real(p)
    import mdtf
    from mdtf.cluster import Server
    from mdtf.train import variables as V
    server = Server.from_env(backend="gloo")
    batch = 4
    Lin, MSE, xs, ys, x_ph, y_ph, Tower, Net = _linear_setup(rank, world, batch)
    base = mdtf.train.AdamOptimizer(0.01)
    tg = []
    tower = Tower(Net(Lin()), "tower_0/", tg, x_ph, y_ph, MSE(), base, batch_size=batch)
    tower.process()
    opt = mdtf.train.SyncReplicasOptimizer(base, world, world, mode="sharded")
    gs = mdtf.train.get_or_create_global_step()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)
    sess = mdtf.train.MonitoredTrainingSession(is_chief=rank == 0, checkpoint_dir=md if rank == 0 else None,
                                               log_step_count_steps=0, server=server, save_checkpoint_secs=None)
    step = gs.value()
    op.reducer.gather_full_master()
    w = {v.name: v.master.tolist() for v in V.get_store().trainable_variables()}
    # this replica's Adam shard, gathered back to full size
    m = op.reducer.gather_full_state(None, "m")[0].tolist()
    with open(os.path.join(out_dir, "resume%d.json" % rank), "w") as f:
        json.dump({"step": step, "weights": w, "adam_m": m, "restored": sess.restored_from}, f)
    sess.close()
    _teardown(server)


def recovery_worker(rank, world, port, steps, out_dir, fault_step=None, fault_task="worker:1", mode="abort",
                    agree="async"):
    """Sync replicas under MonitoredTrainingSession with a chief checkpoint every 2 steps; ``fault_task``
    raises an in-process AbortedError after ``fault_step`` (one replica only): every replica must agree on
    the recovery, restore the chief's checkpoint in process and finish at the same global step."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), MDTF_AGREE=agree)
    import mdtf
    from mdtf.cluster import Server
    from mdtf.cluster.health import FaultInjectionHook
    from mdtf.train import hooks as H
    from mdtf.train import variables as V
    server = Server.from_env(backend="gloo")
    batch = 4
    Lin, MSE, xs, ys, x_ph, y_ph, Tower, Net = _linear_setup(rank, world, batch)
    base = mdtf.train.MomentumOptimizer(0.1, 0.9)
    tg = []
    Tower(Net(Lin()), "tower_0/", tg, x_ph, y_ph, MSE(), base, batch_size=batch).process()
    opt = mdtf.train.SyncReplicasOptimizer(base, replicas_to_aggregate=world, total_num_replicas=world)
    gs = mdtf.train.get_or_create_global_step()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)
    hooks = [H.StopAtStepHook(last_step=steps), opt.make_session_run_hook(rank == 0)]
    if fault_step is not None:
        hooks.append(FaultInjectionHook("worker", rank, step=fault_step, task=fault_task, mode=mode))
    md = os.path.join(out_dir, "model")
    lo, hi = rank * batch, (rank + 1) * batch
    runs = 0
    with mdtf.train.MonitoredTrainingSession(is_chief=rank == 0, checkpoint_dir=md, save_checkpoint_steps=2,
                                             hooks=hooks, log_step_count_steps=0, server=server) as sess:
        while not sess.should_stop():
            sess.run(op, feed_dict={x_ph: xs[lo:hi], y_ph: ys[lo:hi]})
            runs += 1
        rec = sess.recoveries
        agreements = sess.agreements
    w = {v.name: v.master.tolist() for v in V.get_store().trainable_variables()}
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump({"step": gs.value(), "recoveries": rec, "runs": runs, "weights": w, "agreements": agreements}, f)
    _teardown(server)


def fatal_hook_worker(rank, world, port, out_dir):
    """Replica 1's hook raises a non-recoverable ValueError in before_run at global step 3."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import mdtf
    from mdtf.cluster import Server
    from mdtf.train import hooks as H
    server = Server.from_env(backend="gloo")
    batch = 4
    Lin, MSE, xs, ys, x_ph, y_ph, Tower, Net = _linear_setup(rank, world, batch)
    base = mdtf.train.MomentumOptimizer(0.1, 0.9)
    tg = []
    Tower(Net(Lin()), "tower_0/", tg, x_ph, y_ph, MSE(), base, batch_size=batch).process()
    opt = mdtf.train.SyncReplicasOptimizer(base, replicas_to_aggregate=world, total_num_replicas=world)
    gs = mdtf.train.get_or_create_global_step()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)

    class Bug(H.SessionRunHook):
        def before_run(self, rc):
            if rank == 1 and gs.value() == 3:
                raise ValueError("bug in a hook")

    lo, hi = rank * batch, (rank + 1) * batch
    err = None
    sess = mdtf.train.MonitoredTrainingSession(is_chief=rank == 0, hooks=[H.StopAtStepHook(last_step=8), Bug()],
                                               log_step_count_steps=0, server=server)
    try:
        while not sess.should_stop():
            sess.run(op, feed_dict={x_ph: xs[lo:hi], y_ph: ys[lo:hi]})
    except Exception as e:  # noqa: BLE001 - recorded for the test
        err = "%s: %s" % (type(e).__name__, e)
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump({"step": gs.value(), "error": err}, f)
    _teardown(server)


def backup_gpu_worker(rank, world, port, steps, out_dir, replicas):
    """Backup workers on GPU tensors (ranks share the one GPU over gloo): the contributor mask is decided on the
    device from all-gathered clock stamps."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), MDTF_DIST_BACKEND="gloo")
    import mdtf
    from mdtf.cluster import Server
    from mdtf.train import variables as V
    server = Server.from_env(backend="gloo")
    torch.cuda.set_device(0)
    store = V.get_store()
    store.device = torch.device("cuda", 0)
    batch = 4
    Lin, MSE, xs, ys, x_ph, y_ph, Tower, Net = _linear_setup(rank, world, batch)
    base = mdtf.train.MomentumOptimizer(0.1, 0.9)
    tg = []
    Tower(Net(Lin()), "tower_0/", tg, x_ph, y_ph, MSE(), base, batch_size=batch).process()
    opt = mdtf.train.SyncReplicasOptimizer(base, replicas_to_aggregate=replicas, total_num_replicas=world)
    gs = mdtf.train.get_or_create_global_step()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)
    sess = mdtf.train.MonitoredTrainingSession(is_chief=rank == 0, log_step_count_steps=0, server=server,
                                               max_recoveries=0)
    lo, hi = rank * batch, (rank + 1) * batch
    contributed = 0
    for _ in range(steps):
        sess.run(op, feed_dict={x_ph: xs[lo:hi].cuda(), y_ph: ys[lo:hi].cuda()})
        contributed += int(op.last_contributed)
    sess.close()
    w = {v.name: v.master.tolist() for v in V.get_store().trainable_variables()}
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump({"weights": w, "contributed": contributed, "device_mask": bool(op.reducer.backup_device)}, f)
    _teardown(server)


def host_check_worker(rank, world, port, out_dir, fake_hosts):
    """group_is_single_host over a gloo group: real host names (one host) or faked per-rank host names (a
    ClusterSpec job spread over two hosts, where LOCAL_WORLD_SIZE / WORLD_SIZE are not set)."""
    import socket
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for k in ("LOCAL_WORLD_SIZE", "WORLD_SIZE"):
        os.environ.pop(k, None)
    dist.init_process_group("gloo", rank=rank, world_size=world, init_method="tcp://127.0.0.1:%d" % port)
    if fake_hosts:
        socket.gethostname = lambda: "host%d" % (rank % 2)
    from mdtf.parallel.reducer import group_is_single_host
    res = group_is_single_host(None)
    with open(os.path.join(out_dir, "host%d.json" % rank), "w") as f:
        json.dump({"single": res}, f)
    dist.destroy_process_group()
