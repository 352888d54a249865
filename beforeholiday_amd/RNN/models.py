"""RNN constructors (reference: apex/RNN/models.py:8-54)."""
from .cells import GRUCell, LSTMCell, RNNReLUCell, RNNTanhCell, mLSTMRNNCell
from .RNNBackend import RNNCell, bidirectionalRNN, stackedRNN


def toRNNBackend(inputRNN, num_layers, bidirectional=False, dropout=0):
    if bidirectional:
        return bidirectionalRNN(inputRNN, num_layers, dropout=dropout)
    return stackedRNN(inputRNN, num_layers, dropout=dropout)


def LSTM(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0, bidirectional=False,
         output_size=None):
    return toRNNBackend(RNNCell(4, input_size, hidden_size, LSTMCell, 2, bias, output_size), num_layers,
                        bidirectional, dropout=dropout)


def GRU(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0, bidirectional=False,
        output_size=None):
    return toRNNBackend(RNNCell(3, input_size, hidden_size, GRUCell, 1, bias, output_size), num_layers,
                        bidirectional, dropout=dropout)


def ReLU(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0, bidirectional=False,
         output_size=None):
    return toRNNBackend(RNNCell(1, input_size, hidden_size, RNNReLUCell, 1, bias, output_size), num_layers,
                        bidirectional, dropout=dropout)


def Tanh(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0, bidirectional=False,
         output_size=None):
    return toRNNBackend(RNNCell(1, input_size, hidden_size, RNNTanhCell, 1, bias, output_size), num_layers,
                        bidirectional, dropout=dropout)


def mLSTM(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0, bidirectional=False,
          output_size=None):
    return toRNNBackend(mLSTMRNNCell(input_size, hidden_size, bias=bias, output_size=output_size), num_layers,
                        bidirectional, dropout=dropout)
