"""Python RNN stack: LSTM / GRU / ReLU / Tanh / mLSTM (reference: apex/RNN)."""
from .models import GRU, LSTM, ReLU, Tanh, mLSTM

__all__ = ["LSTM", "GRU", "ReLU", "Tanh", "mLSTM", "models"]
