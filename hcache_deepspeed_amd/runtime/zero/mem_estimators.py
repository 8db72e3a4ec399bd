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
             grad_accum_fp32=False, prefetch_depth=2):
    """Returns (gpu_bytes, cpu_bytes) of model states per rank."""
    P, W = float(total_params), max(1, world)
    g = 4.0 if grad_accum_fp32 else 2.0
    lp = 2 * P / W if stage == 3 else 2 * P
    grad = g * P / W if stage >= 2 else g * P
    opt = 12 * P / W if stage >= 1 else 12 * P
    work = 2 * largest_unit_params * (prefetch_depth + 1) if stage == 3 else 0
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
