"""Failure-symmetric setup of communicators that need a collective exchange (symmetric-memory IPC handles, a private
RCCL communicator's unique id).

The hazard it removes: a rank whose LOCAL setup raises (an OOM on a 1 GiB symmetric buffer, an id that could not be
created) used to leave the constructor early and enter the caller's agreement collective, while its peers sat in the
exchange collective of the constructor -- mismatched collectives, i.e. a hang or an exchange of garbage.

Here every rank runs the same collectives whatever happens locally:

1. ``local()`` runs under try/except on every rank and yields (payload to share);
2. ONE ``all_gather_object`` carries (ok, error text, payload) from every rank -- it is the agreement AND the
   exchange; if any rank failed, every rank runs its ``cleanup`` and raises ``CollectiveSetupError`` naming the ranks;
3. ``finish(payloads)`` (open the peers' handles, init the communicator) runs under try/except; ONE more
   ``all_gather_object`` of its ok flags; again either every rank continues or every rank cleans up and raises.

Reference: the reference creates its communicators with a broadcast of the NCCL unique id and no failure agreement
(csrc/compile/deepcompile.cpp:153 via ``init_nccl``; deepspeed/runtime/zero/... symmetric memory through torch).
"""
import torch.distributed as dist


class CollectiveSetupError(RuntimeError):
    """Setup failed on at least one rank of the group; every rank raised it (nothing half-built is kept)."""


def _gather(obj, group):
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [obj]
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


def collective_setup(group, local, finish=None, cleanup=None, what="setup"):
    """Run the three phases above; returns ``(local_result, finish_result)`` on every rank, or raises
    ``CollectiveSetupError`` on every rank. ``local() -> (state, payload)``; ``finish(state, payloads)``;
    ``cleanup(state, finished)`` releases whatever ``local`` / ``finish`` built on this rank (``state`` may be None)."""
    state, payload, err = None, None, ""
    try:
        state, payload = local()
        ok = True
    except Exception as e:  # noqa: BLE001 -- reported to every rank below
        ok, err = False, f"{type(e).__name__}: {e}"[:200]
    everyone = _gather((ok, err, payload), group)
    bad = [(r, e) for r, (o, e, _) in enumerate(everyone) if not o]
    if bad:
        if cleanup is not None and ok:
            cleanup(state, None)
        raise CollectiveSetupError(f"{what}: local setup failed on rank(s) " +
                                   "; ".join(f"{r}: {e}" for r, e in bad))
    fin = None
    if finish is not None:
        err = ""
        try:
            fin = finish(state, [p for _, _, p in everyone])
            ok = True
        except Exception as e:  # noqa: BLE001
            ok, err = False, f"{type(e).__name__}: {e}"[:200]
        agreed = _gather((ok, err), group)
        bad = [(r, e) for r, (o, e) in enumerate(agreed) if not o]
        if bad:
            if cleanup is not None:
                cleanup(state, fin if ok else None)
            raise CollectiveSetupError(f"{what}: exchange failed on rank(s) " +
                                       "; ".join(f"{r}: {e}" for r, e in bad))
    return state, fin
