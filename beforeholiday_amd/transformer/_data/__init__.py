from ._batchsampler import MegatronPretrainingRandomSampler, MegatronPretrainingSampler

__all__ = ["MegatronPretrainingRandomSampler", "MegatronPretrainingSampler"]
