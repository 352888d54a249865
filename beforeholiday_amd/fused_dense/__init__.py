from .fused_dense import (DenseNoBiasFunc, FusedDense, FusedDenseFunc, FusedDenseGeluDense, FusedDenseGeluDenseFunc,
                          dense_no_bias_function, fused_dense_function, fused_dense_gelu_dense_function)
