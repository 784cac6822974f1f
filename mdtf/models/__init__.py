"""Model zoo: LeNet (MNIST), ResNet v1.5 (50/101/152), BERT-base."""
from .lenet import LeNet  # noqa: F401
from .resnet import ResNet, ResNet50, ResNet152, SoftmaxCrossEntropyLoss  # noqa: F401
from .bert import Bert, BertPretrainingLoss, SyntheticBertLoader  # noqa: F401
