"""mdtf — an MI355X-native distributed training framework.

Same capabilities and user API as Seanforfun/Distributed-Tensorflow-Framework
(annotation-configured Model/Loss/Dataloader extension points, ClusterSpec
parameter-server + worker jobs, a between-graph-replication run loop behind a
MonitoredTrainingSession, tf.train.Saver checkpoints), re-designed for AMD
Instinct MI355X (gfx950): PyTorch-ROCm for autograd, hand-written HIP/CDNA4
kernels for the hot ops, RCCL over xGMI for replica synchronisation.
"""
__version__ = "0.1.0"

from . import config, cluster, ops  # noqa: F401
from .config import annotations, flags  # noqa: F401
from .config.flags import FLAGS  # noqa: F401
from . import train  # noqa: F401
from .ops import nn  # noqa: F401
from .train.variables import (get_variable, variable_scope, name_scope, get_variable_scope, AUTO_REUSE,  # noqa: F401
                              add_to_collection, get_collection, trainable_variables, global_variables,
                              GraphKeys, device, reset_default_graph)
from .train.step import placeholder  # noqa: F401
from .cluster import ClusterSpec, Server  # noqa: F401
from . import app  # noqa: F401
from . import estimator  # noqa: F401
from . import errors  # noqa: F401
