from .fmha import FMHA, FMHAFun, fmha_varlen

__all__ = ["FMHA", "FMHAFun", "fmha_varlen"]
