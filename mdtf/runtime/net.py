"""``Net``: wraps a Model with pre/post-process aspects (``distribute_net.py:18-38``)."""
from ..config.annotations import _annotation

# the redundant decorator of distribute_net.py:9-15
current_model = _annotation("current_model", ["net"])


class Net(object):
    def __init__(self, model=None):
        self.model = model

    def inference(self, pre_processed_data):
        assert self.model is not None, "Please either create a model or use annotation @current_model"
        return self.model.inference(pre_processed_data)

    @staticmethod
    def pre_process(input_data, *args, **kwargs):
        return input_data

    @staticmethod
    def post_process(result, *args, **kwargs):
        return result

    def process(self, input_data, *args, **kwargs):
        pre_processed = type(self).pre_process(input_data, *args, **kwargs)
        result = self.inference(pre_processed)
        return type(self).post_process(result, *args, **kwargs)
