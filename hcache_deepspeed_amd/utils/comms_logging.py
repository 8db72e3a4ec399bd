"""Per-collective latency and bandwidth accounting (reference: deepspeed/utils/comms_logging.py).

Bus bandwidth follows the nccl-tests conventions: all_reduce 2(n-1)/n, all_gather/reduce_scatter
(n-1)/n, all_to_all (n-1)/n, point-to-point / broadcast 1. On an 8x MI355X node a ring uses one xGMI
link per direction (~153 GB/s): a busbw much above that means RCCL used several channels/links.
"""
import math

from .logging import logger


def msg_bytes(name, args, kwargs):
    t = None
    if name in ("all_gather_into_tensor", "allgather_fn"):
        t = args[0] if args else kwargs.get("output_tensor")
    elif name in ("reduce_scatter_tensor", "reduce_scatter_fn"):
        t = args[1] if len(args) > 1 else kwargs.get("tensor")
    elif name in ("all_gather", ):
        lst = args[0] if args else kwargs.get("tensor_list")
        return sum(x.numel() * x.element_size() for x in lst)
    elif name in ("reduce_scatter", "all_to_all"):
        lst = args[1] if len(args) > 1 else kwargs.get("input_list", kwargs.get("input_tensor_list"))
        return sum(x.numel() * x.element_size() for x in lst)
    elif name == "all_reduce_coalesced":
        lst = args[0]
        return sum(x.numel() * x.element_size() for x in lst)
    else:
        t = args[0] if args else kwargs.get("tensor")
    if t is None or not hasattr(t, "numel"):
        return 0
    return t.numel() * t.element_size()


def calc_bw(name, size, lat_ms, n):
    if lat_ms <= 0:
        return 0.0, 0.0
    algbw = size / (lat_ms / 1e3)
    if "all_reduce" in name:
        busbw = algbw * 2 * (n - 1) / max(n, 1)
    elif name in ("all_gather_into_tensor", "allgather_fn", "all_gather", "reduce_scatter_tensor",
                  "reduce_scatter_fn", "reduce_scatter", "all_to_all_single", "all_to_all"):
        busbw = algbw * (n - 1) / max(n, 1)
    else:
        busbw = algbw
    return algbw * 8 / 1e9, busbw * 8 / 1e9  # Gbps


def _fmt_size(b):
    if b <= 0:
        return "0B"
    i = int(math.floor(math.log(b, 1024)))
    return f"{b / 1024**i:.2f} {['B', 'KB', 'MB', 'GB', 'TB'][min(i, 4)]}"


class CommsLogger:

    def __init__(self):
        self.enabled = False
        self.prof_all = True
        self.prof_ops = []
        self.verbose = False
        self.debug = False
        self.comms_dict = {}

    def configure(self, enabled, prof_all, prof_ops, verbose, debug):
        self.enabled, self.prof_all, self.prof_ops, self.verbose, self.debug = enabled, prof_all, prof_ops, verbose, debug

    def append(self, raw_name, record_name, latency, msg_size, n):
        if not self.prof_all and record_name not in self.prof_ops:
            return
        algbw, busbw = calc_bw(raw_name, msg_size, latency, n)
        d = self.comms_dict.setdefault(record_name, {})
        ent = d.setdefault(msg_size, [0, [], [], []])
        ent[0] += 1
        ent[1].append(latency)
        ent[2].append(algbw)
        ent[3].append(busbw)
        if self.verbose:
            logger.info(f"comm op: {record_name} | time (ms): {latency:.2f} | msg size: {_fmt_size(msg_size)} | "
                        f"algbw (Gbps): {algbw:.2f} | busbw (Gbps): {busbw:.2f}")

    def log_all(self, print_log=True):
        lines = [f"{'Comm. Op':<24}{'Message Size':<16}{'Count':<8}{'Total Latency(ms)':<20}{'Avg Latency(ms)':<18}"
                 f"{'tput_avg (Gbps)':<18}{'busbw_avg (Gbps)':<18}"]
        for op, sizes in sorted(self.comms_dict.items()):
            for size, (cnt, lats, algs, buss) in sorted(sizes.items()):
                lines.append(f"{op:<24}{_fmt_size(size):<16}{cnt:<8}{sum(lats):<20.2f}{sum(lats) / cnt:<18.2f}"
                             f"{sum(algs) / cnt:<18.2f}{sum(buss) / cnt:<18.2f}")
        if print_log:
            for ln in lines:
                print(ln)
        return lines
