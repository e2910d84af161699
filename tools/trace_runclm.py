"""run_clm under torch.profiler (CPU + GPU activities); writes a chrome trace.
usage: python tools/trace_runclm.py <trace.json> <run_clm args...>"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import run_clm  # noqa: E402


def main():
    out = sys.argv[1]
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                            torch.profiler.ProfilerActivity.CUDA]) as prof:
        run_clm.main(sys.argv[2:])
    prof.export_chrome_trace(out)


if __name__ == "__main__":
    main()
