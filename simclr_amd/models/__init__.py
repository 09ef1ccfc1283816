from .resnet import ResNet, BasicBlock, Bottleneck, resnet18, resnet50, build_backbone
from .heads import (ProjectionHead, LinearClassifier, NonLinearClassifier, CentroidClassifier,
                    Linear)
from .contrastive import ContrastiveModel, SupervisedModel

__all__ = [
    "ResNet", "BasicBlock", "Bottleneck", "resnet18", "resnet50", "build_backbone",
    "ProjectionHead", "LinearClassifier", "NonLinearClassifier", "CentroidClassifier", "Linear",
    "ContrastiveModel", "SupervisedModel",
]
