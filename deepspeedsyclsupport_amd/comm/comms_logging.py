"""Per-collective timing with algbw/busbw (reference `deepspeed/utils/comms_logging.py:34-178`).

Adds an xGMI view: on an 8-GPU MI355X node every GPU has 7 point-to-point links, so the per-link
bandwidth (busbw / 7 for ring-style collectives on the full mesh) is reported next to busbw.
"""
import math

from ..utils.logging import log_dist

XGMI_LINKS = 7


def calc_bw_log(comm_op, size, duration_s, world):
    n = max(world, 1)
    duration_s = max(duration_s, 1e-12)
    if comm_op == "all_to_all_single":
        tput = size / duration_s
        busbw = tput * (n - 1) / n
    elif comm_op in ("all_gather", "all_gather_into_tensor", "reduce_scatter", "reduce_scatter_tensor",
                     "all_gather_coalesced", "reduce_scatter_coalesced"):
        size *= n
        tput = size / duration_s
        busbw = tput * (n - 1) / n
    elif comm_op in ("all_reduce", "all_reduce_coalesced", "inference_all_reduce"):
        tput = size * 2 / duration_s
        busbw = (size / duration_s) * (2 * (n - 1) / n)
    else:
        tput = size / duration_s
        busbw = tput
    # Gbps like the reference
    return tput * 8 / 1e9, busbw * 8 / 1e9


def convert_size(size_bytes):
    if size_bytes == 0:
        return "0B"
    names = ("B", "KB", "MB", "GB", "TB")
    i = int(math.floor(math.log(size_bytes, 1024)))
    return f"{round(size_bytes / 1024**i, 2)} {names[i]}"


class CommsLogger:

    def __init__(self):
        self.comms_dict = {}
        self.verbose = False
        self.debug = False
        self.prof_ops = []
        self.prof_all = True
        self.enabled = False

    def configure(self, cfg):
        self.enabled = cfg.enabled
        self.verbose = cfg.verbose
        self.debug = cfg.debug
        self.prof_ops = list(cfg.prof_ops)
        self.prof_all = cfg.prof_all

    def start_profiling_comms(self):
        self.prof_all = True

    def stop_profiling_comms(self):
        self.prof_all = False

    def append(self, raw_name, record_name, latency_ms, msg_size, world):
        algbw, busbw = calc_bw_log(raw_name, msg_size, latency_ms / 1e3, world)
        d = self.comms_dict.setdefault(record_name, {})
        rec = d.setdefault(msg_size, [0, [], [], []])
        rec[0] += 1
        rec[1].append(latency_ms)
        rec[2].append(algbw)
        rec[3].append(busbw)
        if self.verbose:
            log_dist(f"comm op: {record_name} | time (ms): {latency_ms:.2f} | msg size: {convert_size(msg_size)} | "
                     f"algbw (Gbps): {algbw:.2f} | busbw (Gbps): {busbw:.2f} | per-xGMI-link (GB/s): "
                     f"{busbw / 8 / XGMI_LINKS:.2f}", ranks=[0])

    def log_all(self, print_log=True, show_straggler=False):
        lines = [f"{'Comm. Op':<20}{'Message Size':<20}{'Count':<10}{'Total Latency(ms)':<20}"
                 f"{'Avg Latency(ms)':<20}{'tput_avg (Gbps)':<20}{'busbw_avg (Gbps)':<20}"]
        for op, sizes in sorted(self.comms_dict.items()):
            lines.append(op)
            for sz, (cnt, lats, algs, buss) in sorted(sizes.items()):
                lines.append(f"{' ':<20}{convert_size(sz):<20}{cnt:<10}{sum(lats):<20.2f}{sum(lats) / cnt:<20.2f}"
                             f"{sum(algs) / cnt:<20.2f}{sum(buss) / cnt:<20.2f}")
        out = "\n".join(lines)
        if print_log:
            print(out)
        return out
