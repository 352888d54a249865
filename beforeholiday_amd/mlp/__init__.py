from .mlp import MLP, MlpFunction, mlp_function
