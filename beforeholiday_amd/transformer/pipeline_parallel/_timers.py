"""Named wall-clock timers synchronised with the device (reference: apex/transformer/pipeline_parallel/_timers.py)."""
import time

import torch


def _sync():
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


class _Timer:
    def __init__(self, name):
        self.name_ = name
        self.elapsed_ = 0.0
        self.started_ = False
        self.start_time = time.time()

    def start(self):
        assert not self.started_, "timer has already been started"
        _sync()
        self.start_time = time.time()
        self.started_ = True

    def stop(self):
        assert self.started_, "timer is not started"
        _sync()
        self.elapsed_ += time.time() - self.start_time
        self.started_ = False

    def reset(self):
        self.elapsed_ = 0.0
        self.started_ = False

    def elapsed(self, reset=True):
        started = self.started_
        if started:
            self.stop()
        value = self.elapsed_
        if reset:
            self.reset()
        if started:
            self.start()
        return value


class _Timers:
    def __init__(self):
        self.timers = {}

    def __call__(self, name):
        if name not in self.timers:
            self.timers[name] = _Timer(name)
        return self.timers[name]

    def write(self, names, writer, iteration, normalizer=1.0, reset=False):
        assert normalizer > 0.0
        for name in names:
            writer.add_scalar(name + "-time", self.timers[name].elapsed(reset=reset) / normalizer, iteration)

    def log(self, names, normalizer=1.0, reset=True):
        assert normalizer > 0.0
        string = "time (ms)"
        for name in names:
            string += f" | {name}: {self.timers[name].elapsed(reset=reset) * 1000.0 / normalizer:.2f}"
        if torch.distributed.is_initialized():
            if torch.distributed.get_rank() == torch.distributed.get_world_size() - 1:
                print(string, flush=True)
        else:
            print(string, flush=True)
