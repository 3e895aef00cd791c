#!/usr/bin/env python3
"""Sample socket power and GFX clock of GPU 0 through the amdsmi library (read-only queries, no GPU
compute, no program launched) every 20 ms until SECONDS pass or the file STOP appears; writes one
JSON line: samples, median/max socket W, mean GFX MHz.  Diagnostic only (tools/gpu_slab.sh runs it
beside build_ab/slab's hold mode, so energy per byte = median W / GB/s)."""
import json
import os
import sys
import time


def main():
    seconds, out = float(sys.argv[1]), sys.argv[2]
    stop = sys.argv[3] if len(sys.argv) > 3 else None
    import amdsmi
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    samples = []
    t0 = time.time()
    while time.time() - t0 < seconds and not (stop and os.path.exists(stop)):
        p = amdsmi.amdsmi_get_power_info(h)
        w = p.get("current_socket_power")
        if not isinstance(w, (int, float)) or w <= 0:
            w = p.get("average_socket_power")
        try:
            clk = amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX).get("clk")
        except Exception:
            clk = None
        if isinstance(w, (int, float)) and w > 0:
            samples.append((time.time(), w, clk))
        time.sleep(0.02)
    amdsmi.amdsmi_shut_down()
    ws = sorted(w for _, w, _ in samples)
    cs = [c for _, _, c in samples if isinstance(c, (int, float)) and c > 0]
    rec = {"samples": len(ws), "socket_w_median": ws[len(ws) // 2] if ws else None, "socket_w_max": ws[-1] if ws else None,
           "gfx_mhz_mean": round(sum(cs) / len(cs)) if cs else None, "t0": t0, "t1": time.time(),
           "trace": [(round(t - t0, 3), w, c) for t, w, c in samples]}
    with open(out, "w") as f:
        json.dump(rec, f)


if __name__ == "__main__":
    main()
