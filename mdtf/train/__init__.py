"""tf.train-compatible training API."""
from .optimizer import (Optimizer, GradientDescentOptimizer, MomentumOptimizer, AdamOptimizer,  # noqa: F401
                        AdamWeightDecayOptimizer, SyncReplicasOptimizer)
from .session import Session, MonitoredSession, MonitoredTrainingSession, Scaffold, global_variables_initializer  # noqa: F401,E501
from .hooks import (SessionRunHook, SessionRunArgs, SessionRunContext, SessionRunValues, StopAtStepHook,  # noqa: F401
                    StepCounterHook, CheckpointSaverHook, SummarySaverHook, ExamplesPerSecondHook,
                    LoggingTensorHook, NanTensorHook, ProfilerHook, SecondOrStepTimer, FinalOpsHook)
from .saver import Saver, latest_checkpoint  # noqa: F401
from .device_setter import replica_device_setter, local_device_setter  # noqa: F401
from .variables import get_or_create_global_step, get_global_step, create_global_step  # noqa: F401
from ..data.tfrecord import string_input_producer  # noqa: F401
