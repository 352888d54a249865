from .conv_bias_relu import ConvBias, ConvBiasMaskReLU, ConvBiasReLU, ConvFrozenScaleBiasReLU

__all__ = ["ConvBiasReLU", "ConvBiasMaskReLU", "ConvBias", "ConvFrozenScaleBiasReLU"]
