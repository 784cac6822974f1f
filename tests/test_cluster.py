"""ClusterSpec parsing, rank layout and the done-queue barrier."""
import threading

import pytest

from mdtf.cluster import ClusterSpec, RankLayout, parse_host_list


def test_host_parsing_strips_whitespace():
    # the reference sample had "127.0.0.1: 22" and " 127.0.0.2: 24"
    assert parse_host_list("127.0.0.1:23, 127.0.0.2: 24") == ["127.0.0.1:23", "127.0.0.2:24"]
    assert parse_host_list("") == []
    with pytest.raises(ValueError):
        parse_host_list("localhost")
    with pytest.raises(ValueError):
        parse_host_list("h:99999")


def test_cluster_spec_api():
    c = ClusterSpec({"ps": ["a:1"], "worker": ["b:2", "c:3"]})
    assert c.num_tasks("worker") == 2 and c.num_tasks("ps") == 1
    assert c.task_address("worker", 1) == "c:3"
    assert c.coordinator_address() == "a:1"
    assert ClusterSpec(c) == c
    assert c.as_dict() == {"ps": ["a:1"], "worker": ["b:2", "c:3"]}
    with pytest.raises(ValueError):
        c.task_address("worker", 5)


def test_rank_layout_sync_and_async():
    c = ClusterSpec({"ps": ["h:1", "h:2"], "worker": ["h:3", "h:4", "h:5"]})
    sync = RankLayout(c, gpu_num=2)
    assert sync.world_size == 6 and sync.rank_of("ps", 0) is None
    assert sync.rank_of("worker", 1, 1) == 3
    assert sync.describe(5) == ("worker", 2, 1)
    asy = RankLayout(c, gpu_num=2, async_ps=True)
    assert asy.world_size == 8 and asy.ps_ranks() == [0, 1] and asy.worker_ranks() == list(range(2, 8))
    assert asy.rank_of("worker", 0, 0) == 2
    # GPUs on one host: ps first, then worker towers
    assert asy.local_device_index("ps", 1) == 1
    assert asy.local_device_index("worker", 2, 1) == 2 + 2 * 2 + 1


def test_done_queue_barrier_waits_for_all_workers():
    import datetime
    import torch.distributed as dist
    from mdtf.cluster import launcher
    from mdtf.cluster.server import Server
    port = launcher.free_port()
    c = ClusterSpec({"ps": ["127.0.0.1:%d" % port], "worker": ["127.0.0.1:1", "127.0.0.1:2"]})
    ps = Server(c, "ps", 0, gpu_num=0, async_ps=False)      # hosts the store; joins no collective group
    got = []
    t = threading.Thread(target=lambda: (ps.wait_for_workers(2, timeout_s=20), got.append(True)))
    t.start()
    client = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=20))
    client.add("mdtf/done_queue0", 1)
    assert not got
    client.add("mdtf/done_queue0", 1)
    t.join(10)
    assert got == [True]


def test_backup_clock_refresh_is_host_side_and_restarts_after_restore():
    """The device-clock offsets of the GPU backup-worker path are re-measured on the host between steps (also
    between hipGraph replays), every BACKUP_RECALIBRATE_STEPS global steps; a global step that went back (a
    restore after a recovery) restarts the period instead of re-measuring inside the next capture."""
    from mdtf.parallel.reducer import GradReducer

    class Fake(object):
        BACKUP_RECALIBRATE_STEPS = 10
        backup_device = True
        measured = 0

        def _measure_clock_offsets(self):
            self.measured += 1

    f = Fake()
    f._bk = {"at": None}
    refresh = GradReducer.refresh_backup_clock
    assert refresh(f, 5) is False and f._bk["at"] == 5          # first use sets the period origin
    assert refresh(f, 14) is False and f.measured == 0
    assert refresh(f, 15) is True and f.measured == 1 and f._bk["at"] == 15
    assert refresh(f, 3) is False and f._bk["at"] == 3           # restored to an earlier step: restart
    assert refresh(f, 12) is False and f.measured == 1
    assert refresh(f, 13) is True and f.measured == 2
