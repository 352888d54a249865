from .transducer import TransducerJoint, TransducerLoss

__all__ = ["TransducerJoint", "TransducerLoss"]
