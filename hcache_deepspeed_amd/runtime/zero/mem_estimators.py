"""Model-state memory estimators for the flat-shard ZeRO store.

Reference parity: stage_1_and_2.py ``estimate_zero2_model_states_mem_needs*`` (:2442-2520) and stage3.py
``estimate_zero3_model_states_mem_needs*`` (:3005-3148). The byte counts follow THIS framework's layout:
compute-dtype params (2 B), gradients (2 B, or 4 B fp32 when accumulating), fp32 master (4 B) and Adam moments
(8 B), each divided by the data-parallel size where the stage shards it; ZeRO-3 keeps
(prefetch_depth + 1) gathered units live; offload moves master+moments (and params for ZeRO-Infinity) to host.
"""
from ...utils.logging import logger

GB = 2**30


def model_to_params(model):
    total = sum(dict((id(p), getattr(p, "ds_numel", p.numel())) for p in model.parameters()).values())
    largest = 0
    for m in model.modules():
        largest = max(largest, sum(getattr(p, "ds_numel", p.numel()) for p in m.parameters(recurse=False)))
    return total, largest


def estimate(total_params, stage, world, largest_unit_params=0, offload_optimizer=False, offload_param=False,
             grad_accum_fp32=False, prefetch_depth=2, reduce_inflight=2, root_params=0):
    """Returns (gpu_bytes, cpu_bytes) of model states per rank.

    ZeRO-3 working set at dp>1 (runtime/zero/optimizer.py): (prefetch_depth + 1) gathered units, the current
    unit's unsharded gradient plus ``reduce_inflight`` gradients still in a reduce-scatter, and the persistent
    root unit (embeddings / LM head / final norm: ``root_params``) gathered with its unsharded gradient."""
    P, W = float(total_params), max(1, world)
    g = 4.0 if grad_accum_fp32 else 2.0
    lp = 2 * P / W if stage == 3 else 2 * P
    grad = g * P / W if stage >= 2 else g * P
    opt = 12 * P / W if stage >= 1 else 12 * P
    work = 0
    if stage == 3 and W > 1:
        work = 2 * largest_unit_params * (prefetch_depth + 1) + 2 * largest_unit_params * (1 + reduce_inflight)
        work += 2 * root_params + 2 * root_params
    cpu = 0.0
    if offload_optimizer:
        cpu += opt
        opt = 0.0
    if offload_param and stage == 3:
        cpu += lp
        lp = 0.0
    return int(lp + grad + opt + work), int(cpu)


def _table(rows):
    for r in rows:
        logger.info("  " + " | ".join(r))


def estimate_zero2_model_states_mem_needs(total_params, num_gpus_per_node=1, num_nodes=1, cpu_offload=True,
                                          additional_buffer_factor=1.5):
    gpu, cpu = estimate(total_params, 2, num_gpus_per_node * num_nodes, offload_optimizer=cpu_offload)
    return int(cpu * additional_buffer_factor), gpu


def estimate_zero3_model_states_mem_needs(total_params, largest_layer_params, num_gpus_per_node=1, num_nodes=1,
                                          cpu_offload=True, cpu_offload_params=True, zero_init=True,
                                          additional_buffer_factor=1.5):
    gpu, cpu = estimate(total_params, 3, num_gpus_per_node * num_nodes, largest_layer_params,
                        offload_optimizer=cpu_offload, offload_param=cpu_offload and cpu_offload_params)
    return int(cpu * additional_buffer_factor), gpu, 4 * largest_layer_params


def _all(total, largest, stage, num_gpus_per_node, num_nodes, factor):
    rows = [f"Estimated memory needed for params, optim states and gradients ({num_nodes} node(s) x "
            f"{num_gpus_per_node} GPU(s), {total / 1e6:.0f}M params, ZeRO-{stage}):",
            "per CPU  |  per GPU |   Options"]
    out = []
    opts = [(False, False), (True, False)] + ([(True, True)] if stage == 3 else [])
    for off_opt, off_par in opts:
        gpu, cpu = estimate(total, stage, num_gpus_per_node * num_nodes, largest, off_opt, off_par)
        cpu = int(cpu * factor)
        out.append((cpu, gpu, off_opt, off_par))
        rows.append(f"{cpu / GB:7.2f}GB | {gpu / GB:7.2f}GB | offload_optimizer={'cpu' if off_opt else 'none'}"
                    + (f", offload_param={'cpu' if off_par else 'none'}" if stage == 3 else ""))
    for r in rows:
        print(r)
    return out


def estimate_zero2_model_states_mem_needs_all_live(model, num_gpus_per_node=1, num_nodes=1,
                                                   additional_buffer_factor=1.5):
    total, largest = model_to_params(model)
    return _all(total, largest, 2, num_gpus_per_node, num_nodes, additional_buffer_factor)


def estimate_zero2_model_states_mem_needs_all_cold(total_params, num_gpus_per_node=1, num_nodes=1,
                                                   additional_buffer_factor=1.5):
    return _all(total_params, 0, 2, num_gpus_per_node, num_nodes, additional_buffer_factor)


def estimate_zero3_model_states_mem_needs_all_live(model, num_gpus_per_node=1, num_nodes=1,
                                                   additional_buffer_factor=1.5):
    total, largest = model_to_params(model)
    return _all(total, largest, 3, num_gpus_per_node, num_nodes, additional_buffer_factor)


def estimate_zero3_model_states_mem_needs_all_cold(total_params, largest_layer_params, num_gpus_per_node=1,
                                                   num_nodes=1, additional_buffer_factor=1.5):
    return _all(total_params, largest_layer_params, 3, num_gpus_per_node, num_nodes, additional_buffer_factor)


def llama_activation_bytes(cfg, tokens, ckpt=False):
    """Saved-activation bytes of one micro-batch of ``tokens`` tokens through models/llama.py (bf16, fused
    FlashAttention saving O + LSE, fused SwiGLU saving its input, chunked fused LM-head CE saving nothing
    of size V). Per layer and token: block input, the two RMSNorm outputs, Q|K|V, the attention output,
    the MLP residual input, gate|up and the SwiGLU output (H*6 + 3*I + 2*KV elements). With activation
    checkpointing only the block input survives. Calibrated against the measured 1-GPU bench
    (Llama-3-8B, mb7, seq 4096: 244.5 GiB peak = 119.6 GiB states + ~125 GiB activations/workspace)."""
    H, I = cfg.hidden_size, cfg.intermediate_size
    kv = cfg.num_key_value_heads * cfg.head_dim
    per = H if ckpt else 6 * H + 3 * I + 2 * kv
    return 2 * per * cfg.num_hidden_layers * tokens


def estimate_llama_training(cfg, micro_batch, seq, world, stage=3, prefetch_depth=2, reduce_inflight=2,
                            offload_optimizer=False, offload_param=False, ckpt=False, hbm_gib=268.0):
    """Per-GPU HBM plan for one of the bench configs: model states + ZeRO-3 working set + activations.
    Returns a dict of GiB figures and whether it fits in ``hbm_gib`` (MI355X: 288 GB HBM3E, of which
    torch sees 268 GiB)."""
    H, V, L = cfg.hidden_size, cfg.vocab_size, cfg.num_hidden_layers
    kv = cfg.num_key_value_heads * cfg.head_dim
    layer = H * (cfg.num_attention_heads * cfg.head_dim + 2 * kv) + cfg.num_attention_heads * cfg.head_dim * H \
        + 3 * H * cfg.intermediate_size + 2 * H
    root = V * H * (1 if getattr(cfg, "tie_word_embeddings", False) else 2) + H
    total = layer * L + root
    gpu, cpu = estimate(total, stage, world, layer, offload_optimizer, offload_param, False, prefetch_depth,
                        reduce_inflight, root)
    act = llama_activation_bytes(cfg, micro_batch * seq, ckpt)
    tot = gpu + act
    return {"params_b": total / 1e9, "states_gib": gpu / GB, "activations_gib": act / GB, "total_gib": tot / GB,
            "host_gib": cpu / GB, "fits": tot / GB <= hbm_gib}


def long_context_plan(cfg, n_gpus=8, sp=8, host_ram_gib=2048.0, host_fraction=0.4, hbm_gib=268.0, stash=True,
                      max_tokens=1 << 26):
    """Largest sequence length S one node trains with Ulysses SP + the host activation cache (``ckpt_offload``) and
    ZeRO-3 over all ``n_gpus`` ranks (dp = n_gpus / sp sequences in flight), and what it costs in host DRAM.

    Per rank (S_loc = S / sp tokens):
      * host (pinned): every block's checkpointed boundary (H bf16 per token and layer) and, with ``stash``, its
        attention output + LSE (n_q*d bf16 + n_q fp32) -- ``host_fraction`` of the node's RAM is the pinned budget,
        shared by the node's ranks (offload/activation_cache.default_host_budget_gib);
      * HBM: ZeRO-3 states sharded n_gpus ways + the gathered working set, a fixed workspace (MLP run in 64k-row
        chunks, LM-head CE chunks, copy window: 40 GiB), one block's recompute transients for S_loc tokens
        (~12 H bf16 values per token incl. gradients), and the all-to-all'ed attention of the FULL sequence for this
        rank's n_q/sp heads (q, k, v, o and their gradients).
    Calibration against the one-GPU 512k run (profiles/r5/ckoff512k_r5d.json): the plan's HBM at n_gpus = sp = 1,
    S = 512k is 227.7 GiB (measured peak 221.5 GiB with 10 blocks' stash kept on the device); its host bytes without
    the stash are 128 GiB of boundaries (measured 156.6 GiB pinned: the boundaries plus the stash of the 9 blocks that
    fit the budget -- the cache stashes only what the pinned budget holds, so ``stash`` True / False bracket it).
    Returns {"max_seq": S, "host_gib_node": ..., "hbm_gib_rank": ..., "limited_by": "host" | "hbm"}."""
    H, L = cfg.hidden_size, cfg.num_hidden_layers
    nq, nkv, d = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    gpu_states, _ = estimate(cfg.num_params(include_embedding=True) if hasattr(cfg, "num_params") else 8.03e9, 3,
                             n_gpus, H * (nq * d + 2 * nkv * d) + nq * d * H + 3 * H * cfg.intermediate_size)
    host_per_tok_rank = L * (2 * H + ((2 * nq * d + 4 * nq) if stash else 0))
    lq, lkv = max(1, nq // sp), max(1, nkv // sp)
    full_attn_per_tok = 2 * 2 * (2 * lq + 2 * lkv) * d  # q,k,v,o + grads for this rank's heads over the full S
    dev_per_loc_tok = 12 * 2 * H
    fixed = 40 * GB
    budget_host = host_fraction * host_ram_gib * GB
    dp = max(1, n_gpus // sp)

    def need(S):
        s_loc = S // sp
        host = host_per_tok_rank * s_loc * n_gpus  # every rank of the node holds its slice (dp groups: own sequences)
        dev = gpu_states + fixed + dev_per_loc_tok * s_loc + full_attn_per_tok * S
        return host, dev

    lo, hi = 0, max_tokens
    while hi - lo > 1024:
        mid = (lo + hi) // 2 // 1024 * 1024
        host, dev = need(mid)
        if host <= budget_host and dev <= hbm_gib * GB:
            lo = mid
        else:
            hi = mid
    host, dev = need(lo)
    h2, d2 = need(lo + 1024 * sp)
    return {"max_seq": lo, "n_gpus": n_gpus, "sp": sp, "dp": dp, "host_gib_node": round(host / GB, 1),
            "host_budget_gib_node": round(budget_host / GB, 1), "hbm_gib_rank": round(dev / GB, 1),
            "limited_by": "host" if h2 > budget_host else "hbm", "stash_attention": stash}
