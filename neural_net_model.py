"""Reference-compatible module path: ``from neural_net_model import NeuralNetworkModel, ...``.

The implementation lives in :mod:`penr_oz_neural_network_torch_amd.models`; this module only
re-exports it so code and tests written against the reference (``neural_net_model.py``) run
unchanged.
"""
from penr_oz_neural_network_torch_amd.models import (BatchNormLayer, EmbeddingLayer, FlattenLayer,  # noqa: F401
                                                     Layer, LinearLayer, MultiLayerPerceptron, NeuralNetworkModel,
                                                     ReluLayer, SigmoidLayer, SoftmaxLayer, TanhLayer)

__all__ = ["Layer", "EmbeddingLayer", "FlattenLayer", "LinearLayer", "BatchNormLayer", "SigmoidLayer",
           "ReluLayer", "TanhLayer", "SoftmaxLayer", "MultiLayerPerceptron", "NeuralNetworkModel"]
