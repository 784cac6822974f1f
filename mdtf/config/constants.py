"""Framework constants (reference ``distribute_constants.py:14-20``)."""
# Prefix of per-replica scopes; stripped from summary names (distribute_tower.py:139-143).
TOWER_NAME = 'tower'

# Fraction of an epoch kept in the shuffle queue (distribute_constants.py:20).
MIN_FRACTION_OF_EXAMPLE_IN_QUEUE = 0.05

# Default gradient bucket size for the RCCL reducer.  xGMI rings are per-link
# bound (~153 GB/s/direction); 32 MiB buckets keep each collective well above
# the latency floor (~tens of µs) while leaving enough buckets to overlap with
# backward on ResNet-50 (~100 MB of fp32 grads -> ~4 buckets).
DEFAULT_BUCKET_BYTES = 32 << 20


def bucket_bytes():
    """Bucket size in bytes: ``MDTF_BUCKET_MB`` if set, else DEFAULT_BUCKET_BYTES
    (``bench/collectives.py`` sweeps 4-256 MiB on a node to choose it)."""
    import os
    mb = os.environ.get("MDTF_BUCKET_MB")
    return int(float(mb) * (1 << 20)) if mb else DEFAULT_BUCKET_BYTES

# Rendezvous defaults.
DEFAULT_PORT = 29500
STORE_TIMEOUT_S = 600


def initial_learning_rate():
    """The reference's INITIAL_LEARNING_RATE (read lazily from the flag)."""
    from .flags import FLAGS
    return FLAGS.train_learning_rate
