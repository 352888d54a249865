"""Stacked / bidirectional RNN drivers and the generic RNN cell (reference: apex/RNN/RNNBackend.py:10-365).

Sequence-major ([time, batch, features]); every cell step is one fused torch RNN-cell call
(``torch._VF.lstm_cell`` / ``gru_cell`` / ``rnn_*_cell``: input and recurrent GEMMs on hipBLASLt and
the gate pointwise math in one kernel).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def is_iterable(maybe_iterable):
    return isinstance(maybe_iterable, (list, tuple))


def flatten_list(tens_list):
    """Stack a list of [bsz, features] tensors into [len, bsz, features]."""
    if not is_iterable(tens_list):
        return tens_list
    return torch.cat(tens_list, dim=0).view(len(tens_list), *tens_list[0].size())


class bidirectionalRNN(nn.Module):
    def __init__(self, inputRNN, num_layers=1, dropout=0):
        super().__init__()
        self.dropout = dropout
        self.fwd = stackedRNN(inputRNN, num_layers=num_layers, dropout=dropout)
        self.bckwrd = stackedRNN(inputRNN.new_like(), num_layers=num_layers, dropout=dropout)
        self.rnns = nn.ModuleList([self.fwd, self.bckwrd])

    def forward(self, input, collect_hidden=False):
        fwd_out, fwd_hiddens = self.fwd(input, collect_hidden=collect_hidden)
        bck_out, bck_hiddens = self.bckwrd(input, reverse=True, collect_hidden=collect_hidden)
        output = torch.cat([fwd_out, bck_out], -1)
        hiddens = tuple(torch.cat(h, -1) for h in zip(fwd_hiddens, bck_hiddens))
        return output, hiddens

    def reset_parameters(self):
        for rnn in self.rnns:
            rnn.reset_parameters()

    def init_hidden(self, bsz):
        for rnn in self.rnns:
            rnn.init_hidden(bsz)

    def detach_hidden(self):
        for rnn in self.rnns:
            rnn.detach_hidden()

    def reset_hidden(self, bsz):
        for rnn in self.rnns:
            rnn.reset_hidden(bsz)

    def init_inference(self, bsz):
        for rnn in self.rnns:
            rnn.init_inference(bsz)


class stackedRNN(nn.Module):
    """Layers of one RNNCell type; returns (output [T, B, F], hidden states per kind [layer, B, F]
    (or per time step with ``collect_hidden``))."""

    def __init__(self, inputRNN, num_layers=1, dropout=0):
        super().__init__()
        self.dropout = dropout
        if isinstance(inputRNN, RNNCell):
            rnns = [inputRNN]
            for _ in range(num_layers - 1):
                rnns.append(inputRNN.new_like(inputRNN.output_size))
        elif isinstance(inputRNN, list):
            assert len(inputRNN) == num_layers, "RNN list length must be equal to num_layers"
            rnns = inputRNN
        else:
            raise RuntimeError()
        self.nLayers = len(rnns)
        self.rnns = nn.ModuleList(rnns)

    def forward(self, input, collect_hidden=False, reverse=False):
        seq_len = input.size(0)
        steps = reversed(range(seq_len)) if reverse else range(seq_len)
        hidden_states = [[] for _ in range(self.nLayers)]
        outputs = []
        for t in steps:
            prev = input[t]
            for layer in range(self.nLayers):
                if layer > 0 and self.dropout > 0 and self.training:
                    prev = F.dropout(prev, self.dropout, True)
                outs = self.rnns[layer](prev)
                if collect_hidden or t == (0 if reverse else seq_len - 1):
                    hidden_states[layer].append(outs)
                prev = outs[0]
            outputs.append(prev)
        if reverse:
            outputs = list(reversed(outputs))
        output = flatten_list(outputs)
        n_steps = seq_len if collect_hidden else 1
        n_hid = self.rnns[0].n_hidden_states
        hs = [[[hidden_states[k][j][i] for k in range(self.nLayers)] for j in range(n_steps)] for i in range(n_hid)]
        if reverse:
            hs = [list(reversed(entry)) for entry in hs]
        hs = [[flatten_list(seq) for seq in h] for h in hs]
        if not collect_hidden:
            hs = [entry[0] for entry in hs]
        return output, hs

    def reset_parameters(self):
        for rnn in self.rnns:
            rnn.reset_parameters()

    def init_hidden(self, bsz):
        for rnn in self.rnns:
            rnn.init_hidden(bsz)

    def detach_hidden(self):
        for rnn in self.rnns:
            rnn.detach_hidden()

    def reset_hidden(self, bsz):
        for rnn in self.rnns:
            rnn.reset_hidden(bsz)

    def init_inference(self, bsz):
        for rnn in self.rnns:
            rnn.init_inference(bsz)


class RNNCell(nn.Module):
    """Generic cell: ``gate_multiplier`` (4 LSTM, 3 GRU, 1 plain RNN), optional output projection
    when ``output_size != hidden_size``, hidden state kept across calls (truncated BPTT via
    ``detach_hidden``)."""

    def __init__(self, gate_multiplier, input_size, hidden_size, cell, n_hidden_states=2, bias=False,
                 output_size=None):
        super().__init__()
        self.gate_multiplier = gate_multiplier
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.cell = cell
        self.bias = bias
        self.output_size = hidden_size if output_size is None else output_size
        self.gate_size = gate_multiplier * hidden_size
        self.n_hidden_states = n_hidden_states
        self.w_ih = nn.Parameter(torch.empty(self.gate_size, input_size))
        self.w_hh = nn.Parameter(torch.empty(self.gate_size, self.output_size))
        if self.output_size != hidden_size:
            self.w_ho = nn.Parameter(torch.empty(self.output_size, hidden_size))
        self.b_ih = self.b_hh = None
        if bias:
            self.b_ih = nn.Parameter(torch.empty(self.gate_size))
            self.b_hh = nn.Parameter(torch.empty(self.gate_size))
        self.hidden = [None for _ in range(n_hidden_states)]
        self.reset_parameters()

    def new_like(self, new_input_size=None):
        return type(self)(self.gate_multiplier, self.input_size if new_input_size is None else new_input_size,
                          self.hidden_size, self.cell, self.n_hidden_states, self.bias, self.output_size)

    def reset_parameters(self, gain=1):
        stdev = 1.0 / math.sqrt(self.hidden_size)
        for p in self.parameters():
            p.data.uniform_(-stdev, stdev)

    def init_hidden(self, bsz):
        ref = next(self.parameters())
        for i in range(len(self.hidden)):
            if self.hidden[i] is None or self.hidden[i].size(0) != bsz:
                size = self.output_size if i == 0 else self.hidden_size
                self.hidden[i] = ref.new_zeros(bsz, size)

    def reset_hidden(self, bsz):
        self.hidden = [None for _ in self.hidden]
        self.init_hidden(bsz)

    def detach_hidden(self):
        for i in range(len(self.hidden)):
            if self.hidden[i] is None:
                raise RuntimeError("Must initialize hidden state before you can detach it")
        self.hidden = [h.detach() for h in self.hidden]

    def init_inference(self, bsz):
        self.reset_hidden(bsz)

    def forward(self, input):
        self.init_hidden(input.size(0))
        hidden_state = self.hidden[0] if self.n_hidden_states == 1 else tuple(self.hidden)
        out = self.cell(input, hidden_state, self.w_ih, self.w_hh, b_ih=self.b_ih, b_hh=self.b_hh)
        self.hidden = list(out) if self.n_hidden_states > 1 else [out]
        if self.output_size != self.hidden_size:
            self.hidden[0] = F.linear(self.hidden[0], self.w_ho)
        return tuple(self.hidden)
