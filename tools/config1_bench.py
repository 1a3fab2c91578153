"""Config 1 timing (BASELINE.json configs[0]): oracle/ws_echo.c's echo pair
over 127.0.0.1, stock build (the reference codec) beside the drop-in build
(libcfws.so in place of co_ws_frame.c / co_ws_config.c), both under the
reference's own callers. Test infrastructure: it runs binaries under
oracle/_ref and is not bench.py's measured path.

    python tools/config1_bench.py --out gpurun_out/config1.jsonl
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from echo_util import free_port, run_echo  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--frames", type=int, default=100_000)
    ap.add_argument("--latency-frames", type=int, default=20_000)
    ap.add_argument("--payload", type=int, default=1024)
    ap.add_argument("--modes", default="ws,h2")
    ap.add_argument("--builds", default="stock,cfws,cfws:device",
                    help="cfws:device = the drop-in build with CFWS_DROPIN_GPU_MIN=0 (every "
                         "masked payload to the device)")
    ap.add_argument("--windows", default="64,1")
    a = ap.parse_args()
    with open(a.out, "a") as f:
        for mode in a.modes.split(","):
            for window in [int(w) for w in a.windows.split(",")]:
                frames = a.frames if window > 1 else a.latency_frames
                for rep in range(a.reps):
                    port = free_port()
                    for spec in a.builds.split(","):
                        build, _, pol = spec.partition(":")
                        env = {"CFWS_DROPIN_GPU_MIN": "0"} if pol == "device" else None
                        r = run_echo(build, mode, frames, a.payload, window=window, seed=1, port=port,
                                     timeout=600, env=env)
                        line = {"build": spec, "rep": rep, "client_rc": r["client_rc"],
                                **(r["client"] or {"mode": mode, "window": window, "error": r["client_err"]})}
                        f.write(json.dumps(line) + "\n")
                        f.flush()
                        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
