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



class NebulaCheckpointEngine(AsyncCheckpointEngine):
    """Tiered asynchronous checkpointing with the reference Nebula config (nebula/config.py: ``enabled``,
    ``persistent_storage_path``, ``persistent_time_interval``, ``num_of_version_in_retention``,
    ``enable_nebula_load``, ``load_path``).

    Azure's Nebula service is replaced by the same two tiers on local resources: ``save`` writes each file to the
    fast tier (the checkpoint directory) asynchronously from pinned host copies; every
    ``persistent_time_interval``-th ``commit`` additionally copies the tag's files to ``persistent_storage_path``
    in a background thread, keeping the newest ``num_of_version_in_retention`` tags there. ``load`` prefers the fast
    tier and falls back to the persistent one when ``enable_nebula_load`` is set."""

    def __init__(self, config_params=None):
        super().__init__(config_params)
        cfg = dict(getattr(config_params, "nebula", None) or (config_params or {}) if isinstance(
            config_params, dict) else getattr(config_params, "nebula", None) or {})
        self.persistent_path = cfg.get("persistent_storage_path")
        self.interval = max(1, int(cfg.get("persistent_time_interval", 100) or 1))
        self.retention = max(1, int(cfg.get("num_of_version_in_retention", 2) or 1))
        self.enable_load = bool(cfg.get("enable_nebula_load", True))
        self.load_path = cfg.get("load_path")
        self._written = {}
        self._commits = 0
        self._persist_threads = []
        self._persisted = []

    def save(self, state_dict, path):
        self._written.setdefault(self._tag, []).append(path)
        super().save(state_dict, path)

    def _persist(self, tag, files, prev=None):
        import shutil
        if prev is not None:  # persist in commit order, so retention always drops the OLDEST tags
            prev.join()
        dst = os.path.join(self.persistent_path, str(tag))
        os.makedirs(dst, exist_ok=True)
        for f in files:
            shutil.copy2(f, os.path.join(dst, os.path.basename(f)))
        self._persisted.append(dst)
        while len(self._persisted) > self.retention:
            shutil.rmtree(self._persisted.pop(0), ignore_errors=True)

    def commit(self, tag):
        super().commit(tag)
        files = self._written.pop(tag, [])
        self._commits += 1
        if self.persistent_path and files and self._commits % self.interval == 0:
            prev = self._persist_threads[-1] if self._persist_threads else None
            t = threading.Thread(target=self._persist, args=(tag, files, prev), daemon=False)
            t.start()
            self._persist_threads.append(t)
        return True

    def wait_persisted(self):
        for t in self._persist_threads:
            t.join()
        self._persist_threads = []

    def load(self, path, map_location=None):
        if os.path.exists(path) or not (self.enable_load and (self.load_path or self.persistent_path)):
            return super().load(path, map_location)
        base = self.load_path or self.persistent_path
        tag = os.path.basename(os.path.dirname(path))
        return super().load(os.path.join(base, tag, os.path.basename(path)), map_location)
