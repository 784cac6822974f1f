"""TF-named error classes (``tf.errors``) raised by the mdtf runtime.

``MonitoredSession`` treats :class:`AbortedError` and :class:`UnavailableError` as recoverable:
the session is re-created in the same process (checkpoint restore) and the step is retried, as
TF's ``_RecoverableSession`` does (reference ``distribute_train.py:169-180`` runs its loop under
``MonitoredTrainingSession``).  Store (rendezvous) connection failures and timeouts surface as
:class:`UnavailableError`.
"""


class OpError(RuntimeError):
    def __init__(self, node_def=None, op=None, message=""):
        super(OpError, self).__init__(message)
        self.node_def = node_def
        self.op = op
        self.message = message


class AbortedError(OpError):
    """The operation was aborted (e.g. a concurrency conflict or an injected abort)."""


class UnavailableError(OpError):
    """A service (the cluster store, a peer) is temporarily unreachable."""


class DeadlineExceededError(OpError):
    pass


class InvalidArgumentError(OpError):
    pass


class NotFoundError(OpError):
    pass


RECOVERABLE = (AbortedError, UnavailableError)


def as_recoverable(exc):
    """Map a transient low-level exception to a TF error class, or None if it is not recoverable.

    torch.distributed store failures (``DistStoreError``, ``DistNetworkError``, store timeouts) are
    transient from the session's point of view: the store is re-contacted when the session is re-created.
    """
    if isinstance(exc, RECOVERABLE):
        return exc
    names = {type(exc).__name__} | {c.__name__ for c in type(exc).__mro__}
    if names & {"DistStoreError", "DistNetworkError"}:
        return UnavailableError(message=str(exc))
    return None
