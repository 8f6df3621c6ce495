"""Reference-compatible model API: layers (L2), MLP builder (L3), ``NeuralNetworkModel`` (L4/L5)."""
from .layers import (BatchNormLayer, EmbeddingLayer, FlattenLayer, Layer, LinearLayer, ReluLayer,  # noqa: F401
                     SigmoidLayer, SoftmaxLayer, TanhLayer)
from .mlp import MultiLayerPerceptron, normalize_algos  # noqa: F401
from .network import NeuralNetworkModel  # noqa: F401

__all__ = ["Layer", "EmbeddingLayer", "FlattenLayer", "LinearLayer", "BatchNormLayer", "SigmoidLayer", "ReluLayer",
           "TanhLayer", "SoftmaxLayer", "MultiLayerPerceptron", "NeuralNetworkModel", "normalize_algos"]
