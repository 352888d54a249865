"""Cell functions and the multiplicative LSTM (reference: apex/RNN/cells.py:12-84)."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .RNNBackend import RNNCell


def _lstm_pointwise(input, h_in, cx, w_ih, w_hh, b_ih, b_hh):
    gates = F.linear(input, w_ih, b_ih) + F.linear(h_in, w_hh, b_hh)
    i, f, g, o = gates.chunk(4, 1)
    cy = torch.sigmoid(f) * cx + torch.sigmoid(i) * torch.tanh(g)
    return torch.sigmoid(o) * torch.tanh(cy), cy


def LSTMCell(input, hidden, w_ih, w_hh, b_ih=None, b_hh=None):
    hx, cx = hidden
    if hx.size(1) != cx.size(1):  # recurrent projection: h and c differ in width
        return _lstm_pointwise(input, hx, cx, w_ih, w_hh, b_ih, b_hh)
    return torch._VF.lstm_cell(input, hidden, w_ih, w_hh, b_ih, b_hh)


def GRUCell(input, hidden, w_ih, w_hh, b_ih=None, b_hh=None):
    return torch._VF.gru_cell(input, hidden, w_ih, w_hh, b_ih, b_hh)


def RNNReLUCell(input, hidden, w_ih, w_hh, b_ih=None, b_hh=None):
    return torch._VF.rnn_relu_cell(input, hidden, w_ih, w_hh, b_ih, b_hh)


def RNNTanhCell(input, hidden, w_ih, w_hh, b_ih=None, b_hh=None):
    return torch._VF.rnn_tanh_cell(input, hidden, w_ih, w_hh, b_ih, b_hh)


def mLSTMCell(input, hidden, w_ih, w_hh, w_mih, w_mhh, b_ih=None, b_hh=None):
    """Multiplicative LSTM: m = (W_mi x) * (W_mh h); gates from (x, m) through the fused LSTM cell."""
    hx, cx = hidden
    m = F.linear(input, w_mih) * F.linear(hx, w_mhh)
    if m.size(1) != cx.size(1):
        return _lstm_pointwise(input, m, cx, w_ih, w_hh, b_ih, b_hh)
    return torch._VF.lstm_cell(input, (m, cx), w_ih, w_hh, b_ih, b_hh)


class mLSTMRNNCell(RNNCell):
    def __init__(self, input_size, hidden_size, bias=False, output_size=None):
        super().__init__(4, input_size, hidden_size, mLSTMCell, n_hidden_states=2, bias=bias,
                         output_size=output_size)
        self.w_mih = nn.Parameter(torch.empty(self.output_size, self.input_size))
        self.w_mhh = nn.Parameter(torch.empty(self.output_size, self.output_size))
        self.reset_parameters()

    def forward(self, input):
        self.init_hidden(input.size(0))
        self.hidden = list(self.cell(input, tuple(self.hidden), self.w_ih, self.w_hh, self.w_mih, self.w_mhh,
                                     b_ih=self.b_ih, b_hh=self.b_hh))
        if self.output_size != self.hidden_size:
            self.hidden[0] = F.linear(self.hidden[0], self.w_ho)
        return tuple(self.hidden)

    def new_like(self, new_input_size=None):
        return type(self)(self.input_size if new_input_size is None else new_input_size, self.hidden_size, self.bias,
                          self.output_size)
