"""Curriculum learning, data sampler, random-LTD, progressive layer drop, eigenvalue, MoQ (reference
tests/unit/runtime/test_data_efficiency.py, test_pld.py, test_ds_config... strategies)."""
import os

import numpy as np
import pytest
import torch


def test_curriculum_schedules():
    from hcache_deepspeed_amd.runtime.data_pipeline import CurriculumScheduler
    lin = CurriculumScheduler({"min_difficulty": 8, "max_difficulty": 64, "schedule_type": "fixed_linear",
                               "schedule_config": {"total_curriculum_step": 10, "difficulty_step": 8}})
    vals = [lin.update_difficulty(s) for s in range(0, 13)]
    assert vals[0] == 8 and vals[-1] == 64 and all(a <= b for a, b in zip(vals, vals[1:]))
    assert all(v % 8 == 0 for v in vals)
    root = CurriculumScheduler({"min_difficulty": 8, "max_difficulty": 64, "schedule_type": "fixed_root",
                                "schedule_config": {"total_curriculum_step": 10, "difficulty_step": 8,
                                                    "root_degree": 2}})
    assert root.get_difficulty(3) >= lin.get_difficulty(3)
    disc = CurriculumScheduler({"min_difficulty": 1, "max_difficulty": 3, "schedule_type": "fixed_discrete",
                                "schedule_config": {"difficulty": [1, 2, 3], "max_step": [5, 10]}})
    assert [disc.get_difficulty(s) for s in (1, 5, 6, 10, 11)] == [1, 1, 2, 2, 3]


def test_data_sampler_respects_difficulty():
    from hcache_deepspeed_amd.runtime.data_pipeline import DeepSpeedDataSampler
    metric = np.arange(1000) % 100  # difficulty 0..99
    s = DeepSpeedDataSampler(metric, 32, 8, 0, 2, {"min_difficulty": 10, "max_difficulty": 100,
                                                   "schedule_type": "fixed_linear",
                                                   "schedule_config": {"total_curriculum_step": 5,
                                                                       "difficulty_step": 10}})
    it = iter(s)
    first = [next(it) for _ in range(2)]  # rank 0's two micro-batches of step 1
    assert all(metric[i] <= 28 for mb in first for i in mb)
    sd = s.state_dict()
    s2 = DeepSpeedDataSampler(metric, 32, 8, 0, 2)
    s2.load_state_dict(sd)
    assert s2.consumed_samples == 32


def test_random_ltd_gather_scatter_and_layer():
    from hcache_deepspeed_amd.runtime.data_pipeline import (RandomLayerTokenDrop, RandomLTDScheduler, gpt_sample_tokens,
                                                            token_gather, token_scatter)
    x = torch.randn(2, 16, 8)
    idx = gpt_sample_tokens(6, 16, 2)[0]
    assert (idx[:, 1:] > idx[:, :-1]).all()
    part = token_gather(x, idx)
    assert torch.equal(part[1, 3], x[1, idx[1, 3]])
    y = token_scatter(x, part * 2, idx)
    mask = torch.zeros(2, 16, dtype=torch.bool)
    mask[torch.arange(2)[:, None], idx] = True
    assert torch.allclose(y[mask], x[mask] * 2) and torch.equal(y[~mask], x[~mask])
    sch = RandomLTDScheduler({"min_value": 4, "max_value": 16, "schedule_config": {"require_steps": 10,
                                                                                  "seq_per_step": 4}})
    layer = RandomLayerTokenDrop(torch.nn.Linear(8, 8), sch)
    layer.train()
    out = layer(x)
    assert out.shape == x.shape and (out == x).all(-1).sum() >= 2 * (16 - 4)
    assert sch.update_seq(10) == 16


def test_pld_and_engine_curriculum():
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.runtime.progressive_layer_drop import ProgressiveLayerDrop
    p = ProgressiveLayerDrop(theta=0.5, gamma=0.1)
    p.update_state(10)
    assert 0.5 < p.get_theta() < 1.0
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=os.environ.get("MASTER_PORT", "29641"))
    seen = []

    class M(torch.nn.Module):

        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(4, 4)

        def forward(self, x, labels=None, progressive_layer_drop=False, pld_theta=1.0):
            seen.append((x.shape[1], pld_theta))
            return self.lin(x.float()).sum()

    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
           "curriculum_learning": {"enabled": True, "curriculum_type": "seqlen", "min_difficulty": 2,
                                   "max_difficulty": 8, "schedule_type": "fixed_linear",
                                   "schedule_config": {"total_curriculum_step": 3, "difficulty_step": 2}},
           "progressive_layer_drop": {"enabled": True, "theta": 0.5, "gamma": 0.5}}
    eng, _, _, _ = ds.initialize(model=M(), config=cfg)
    for _ in range(4):
        x = torch.randn(2, 8, 4)
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
    lens = [s for s, _ in seen]
    assert lens[0] < 8 and lens[-1] == 8 and lens == sorted(lens)
    assert seen[0][1] == 1.0 and seen[-1][1] < 1.0


def test_eigenvalue_quadratic():
    from hcache_deepspeed_amd.runtime.eigenvalue import Eigenvalue
    torch.manual_seed(0)
    lin = torch.nn.Linear(4, 1, bias=False)
    A = torch.diag(torch.tensor([5.0, 1.0, 0.5, 0.1]))
    w = lin.weight
    loss = 0.5 * (w @ A @ w.t()).sum()
    ev = Eigenvalue(max_iter=200, tol=1e-6)
    res = ev.compute_eigenvalue(torch.nn.ModuleList([lin]), loss=loss)
    assert res[0][0] == pytest.approx(1.0)  # normalised by the max
    ev2 = Eigenvalue(max_iter=200, tol=1e-6)
    ev2.post_process = lambda d: d
    raw = ev2.compute_eigenvalue(torch.nn.ModuleList([lin]), loss=0.5 * (w @ A @ w.t()).sum())
    assert raw[0][0] == pytest.approx(5.0, rel=1e-3)


def test_moq_quantizer_schedule():
    from hcache_deepspeed_amd.runtime.quantize import Quantizer
    p = torch.nn.Parameter(torch.randn(16, 16))
    p.start_bits, p.target_bits, p.q_period = 8, 4, 2
    q = Quantizer(q_groups=4)
    orig = p.data.clone()
    for _ in range(6):
        q.quantize([[p]], overflow=False)
    assert p.start_bits == 4 or p.start_bits < 8
    assert p.data.unique().numel() <= 4 * 2**8
    assert (p.data - orig).abs().max() < orig.abs().max()


# ---- data-sampling tools: indexed dataset, data analyzer, variable batch size + LR ----------------------------
def _write_ref_index(prefix, dtype_code, sizes, doc_idx, items, np_dtype):
    """Writes the reference's documented .idx/.bin layout independently of the framework's builder."""
    import struct
    with open(prefix + ".bin", "wb") as f:
        for it in items:
            f.write(np.asarray(it, dtype=np_dtype).tobytes())
    with open(prefix + ".idx", "wb") as f:
        f.write(b"MMIDIDX\x00\x00")
        f.write(struct.pack("<Q", 1))
        f.write(struct.pack("<B", dtype_code))
        f.write(struct.pack("<Q", len(sizes)))
        f.write(struct.pack("<Q", len(doc_idx)))
        f.write(np.asarray(sizes, np.int32).tobytes())
        ptr = np.concatenate([[0], np.cumsum(np.asarray(sizes[:-1], np.int64) * np.dtype(np_dtype).itemsize)])
        f.write(ptr.astype(np.int64).tobytes())
        f.write(np.asarray(doc_idx, np.int64).tobytes())


def test_mmap_indexed_dataset_roundtrip_and_format(tmp_path):
    from hcache_deepspeed_amd.runtime.data_pipeline.data_sampling import MMapIndexedDataset, make_builder
    items = [np.arange(n, dtype=np.int32) * (n + 1) for n in (3, 0, 7, 1)]
    # our builder -> our reader
    b = make_builder(str(tmp_path / "a.bin"), dtype=np.int32)
    for it in items[:2]:
        b.add_item(torch.from_numpy(it))
    b.end_document()
    for it in items[2:]:
        b.add_item_numpy(it)
    b.end_document()
    b.finalize(str(tmp_path / "a.idx"))
    ds = MMapIndexedDataset(str(tmp_path / "a"))
    assert len(ds) == 4 and list(ds.sizes) == [3, 0, 7, 1] and list(ds.doc_idx) == [0, 2, 4]
    for i, it in enumerate(items):
        assert np.array_equal(ds[i], it)
    assert np.array_equal(ds.get(2, offset=2, length=3), items[2][2:5])
    assert [x.tolist() for x in ds[1:3]] == [items[1].tolist(), items[2].tolist()]
    # byte-identical to an independently written file of the reference layout
    _write_ref_index(str(tmp_path / "r"), 4, [3, 0, 7, 1], [0, 2, 4], items, np.int32)
    assert (tmp_path / "r.idx").read_bytes() == (tmp_path / "a.idx").read_bytes()
    assert (tmp_path / "r.bin").read_bytes() == (tmp_path / "a.bin").read_bytes()
    # merge
    b2 = make_builder(str(tmp_path / "m.bin"), dtype=np.int32)
    b2.merge_file_(str(tmp_path / "a"))
    b2.merge_file_(str(tmp_path / "r"))
    b2.finalize(str(tmp_path / "m.idx"))
    m = MMapIndexedDataset(str(tmp_path / "m"))
    assert len(m) == 8 and list(m.doc_idx) == [0, 2, 4, 6, 8] and np.array_equal(m[6], items[2])


class _TokDataset(torch.utils.data.Dataset):

    def __init__(self, n=97, seed=0):
        g = np.random.default_rng(seed)
        self.lens = g.integers(1, 40, n)
        self.items = [torch.from_numpy(g.integers(0, 50, L)) for L in self.lens]

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]


def _seqlen(batch):
    return np.array([len(x) for x in batch], dtype=np.int64)


def _vocab_hist(batch):
    h = np.zeros(50, dtype=np.int64)
    for x in batch:
        h += np.bincount(x.numpy(), minlength=50)
    return h


@pytest.mark.parametrize("workers,threads", [(1, 1), (2, 3)])
def test_data_analyzer_outputs(tmp_path, workers, threads):
    from hcache_deepspeed_amd.runtime.data_pipeline.data_sampling import DataAnalyzer, MMapIndexedDataset
    from hcache_deepspeed_amd.runtime.data_pipeline.data_sampling.data_analyzer import load_sample_to_metric
    ds = _TokDataset()
    for w in range(workers):
        a = DataAnalyzer(ds, num_workers=workers, worker_id=w, num_threads=threads, batch_size=5,
                         metric_names=["seqlen", "vocab"], metric_functions=[_seqlen, _vocab_hist],
                         metric_types=["single_value_per_sample", "accumulate_value_over_samples"],
                         metric_dtypes=[np.int64, np.int64], save_path=str(tmp_path), collate_fn=lambda b: b)
        a.run_map()
    a.run_reduce()
    s2m = load_sample_to_metric(str(tmp_path), "seqlen")
    assert np.array_equal(s2m, ds.lens)
    d = tmp_path / "seqlen"
    i2m = MMapIndexedDataset(str(d / "seqlen_index_to_metric"))
    i2s = MMapIndexedDataset(str(d / "seqlen_index_to_sample"))
    vals = [int(x[0]) for x in i2m[0:len(i2m)]]
    assert vals == sorted(set(ds.lens.tolist()))
    for v, samples in zip(vals, i2s[0:len(i2s)]):
        assert sorted(samples.tolist()) == sorted(np.nonzero(ds.lens == v)[0].tolist())
    merged = MMapIndexedDataset(str(d / "seqlen_index_to_sample_percentile_merged"))
    assert sorted(np.concatenate(merged[0:len(merged)]).tolist()) == list(range(len(ds)))
    vh = MMapIndexedDataset(str(tmp_path / "vocab" / "vocab_metric_value"))
    assert np.array_equal(vh[0], sum(np.bincount(x.numpy(), minlength=50) for x in ds.items))


def _dist_analyzer(rank, world, path):
    from hcache_deepspeed_amd.runtime.data_pipeline.data_sampling import DistributedDataAnalyzer
    from hcache_deepspeed_amd.runtime.data_pipeline.data_sampling.data_analyzer import load_sample_to_metric
    ds = _TokDataset()
    DistributedDataAnalyzer(ds, batch_size=4, metric_names=["seqlen"], metric_functions=[_seqlen],
                            metric_types=["single_value_per_sample"], save_path=path, collate_fn=lambda b: b,
                            metric_dtypes=[np.int64]).run_map_reduce()
    if rank == 0:
        assert np.array_equal(load_sample_to_metric(path, "seqlen"), ds.lens)


def test_distributed_data_analyzer_world2(tmp_path):
    from tests.dist_utils import run_distributed
    run_distributed(_dist_analyzer, 2, str(tmp_path))


def test_batch_by_seqlens_and_lr_scaling():
    from hcache_deepspeed_amd.runtime.data_pipeline.data_sampling import (batch_by_seqlens,
                                                                          get_dataloader_and_lr_scheduler_for_variable_batch_size,
                                                                          scale_lr)
    ds = _TokDataset(n=200, seed=3)
    mb, sizes, maxlens = batch_by_seqlens(ds.lens, max_tokens=64, effective_batch_size=2,
                                          sequence_picking_order="seqlen")
    assert len(mb) == 2 * len(sizes)
    seen = set()
    for b, ids in mb:
        assert sum(ds.lens[i] for i in ids) <= 64
        assert not (seen & set(ids))
        seen |= set(ids)
        assert max(ds.lens[i] for i in ids) <= maxlens[b]
    assert all(sizes[b] == sum(len(ids) for bb, ids in mb if bb == b) for b in range(len(sizes)))
    mb2, _, _ = batch_by_seqlens(ds.lens, 64, max_batch_size=3, effective_batch_size=1,
                                 required_microbatches_of_same_size=True)
    assert all(len(ids) <= 3 for _, ids in mb2)
    assert scale_lr(8, 16, 1e-3, "linear") == pytest.approx(2e-3)
    assert scale_lr(8, 32, 1e-3, "sqrt") == pytest.approx(2e-3)
    model = torch.nn.Linear(4, 4)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    loader, sched = get_dataloader_and_lr_scheduler_for_variable_batch_size(
        ds, ds.lens, max_tokens=64, effective_batch_size=1, optimizer=opt, dataloader_num_workers=0)
    first = next(iter(loader))
    assert isinstance(first, list) and sum(len(x) for x in first) <= 64
    lrs = []
    for _ in range(3):
        lrs.append(opt.param_groups[0]["lr"])
        sched.step()
    bs = sched.batch_sizes
    assert lrs[0] == pytest.approx(0.1 * bs[0] / 64) and lrs[1] == pytest.approx(0.1 * bs[1] / 64)
    sd = sched.state_dict()
    assert sd["batch_sizes"] == bs


def test_sampler_from_analyzer_output(tmp_path):
    from hcache_deepspeed_amd.runtime.data_pipeline import DataAnalyzer, DeepSpeedDataSampler
    ds = _TokDataset()
    DataAnalyzer(ds, batch_size=8, metric_names=["seqlen"], metric_functions=[_seqlen],
                 metric_types=["single_value_per_sample"], metric_dtypes=[np.int64], save_path=str(tmp_path),
                 collate_fn=lambda b: b).run_map_reduce()
    s = DeepSpeedDataSampler.from_analyzer(str(tmp_path), "seqlen", 8, 4, curriculum_config={
        "min_difficulty": 10, "max_difficulty": 40, "schedule_type": "fixed_linear",
        "schedule_config": {"total_curriculum_step": 10, "difficulty_step": 1}})
    first = next(iter(s))
    assert all(ds.lens[i] <= 13 or ds.lens[i] <= sorted(ds.lens)[7] for i in first)
