from .model import Model, Loss  # noqa: F401
from .net import Net  # noqa: F401
from .tower import Tower  # noqa: F401
from .train import Train  # noqa: F401
from .eval import Eval  # noqa: F401
