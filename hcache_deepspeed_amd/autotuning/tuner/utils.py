"""Tuning-space helpers (reference autotuning/tuner/utils.py: ``dict_to_dims``, ``gen_combinations``, ``flatten``,
``dict_to_feature``)."""
import itertools
import numbers


def gen_combinations(space):
    """A nested dict whose list-valued leaves are choices -> every concrete dict (cartesian product)."""
    keys, choices = [], []

    def walk(d, prefix):
        for k, v in d.items():
            if isinstance(v, dict):
                walk(v, prefix + (k, ))
            else:
                keys.append(prefix + (k, ))
                choices.append(v if isinstance(v, list) else [v])

    walk(space, ())
    for combo in itertools.product(*choices):
        out = {}
        for path, val in zip(keys, combo):
            cur = out
            for p in path[:-1]:
                cur = cur.setdefault(p, {})
            cur[path[-1]] = val
        yield out


def dict_to_dims(space):
    """Number of choices of every list-valued leaf, in traversal order."""
    dims = []

    def walk(d):
        for v in d.values():
            if isinstance(v, dict):
                walk(v)
            elif isinstance(v, list):
                dims.append(len(v))

    walk(space)
    return dims


def flatten(d, parent_key="", sep="_"):
    out = {}
    for k, v in d.items():
        key = f"{parent_key}{sep}{k}" if parent_key else str(k)
        if isinstance(v, dict):
            out.update(flatten(v, key, sep))
        else:
            out[key] = v
    return out


def dict_to_feature(feature_dict, keys, max_value=None):
    """Numeric feature vector of a (flattened) config over ``keys``; booleans -> 0/1, missing -> 0."""
    vec = []
    for k in keys:
        v = feature_dict.get(k, 0)
        if isinstance(v, bool):
            v = float(v)
        elif not isinstance(v, numbers.Number):
            v = 0.0
        if max_value is not None and max_value.get(k):
            v = v / max_value[k]
        vec.append(float(v))
    return vec


def merge_dicts(base, override):
    out = dict(base)
    for k, v in override.items():
        out[k] = merge_dicts(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out
