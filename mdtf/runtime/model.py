"""Model / Loss extension points (``distribute_model.py:13-22``, ``distribute_loss.py:11-19``)."""
import abc


class Model(metaclass=abc.ABCMeta):
    @abc.abstractmethod
    def inference(self, input_data):
        """Forward pass: ``input_data`` (NHWC tensor for images) -> logits.

        Build it from :mod:`mdtf.layers.tools` (or any mdtf/torch ops); variables
        created through ``get_variable`` are shared across steps and replicas.
        """


class Loss(metaclass=abc.ABCMeta):
    @abc.abstractmethod
    def loss(self, predict, ground_truth):
        """Return a scalar loss tensor."""
