"""Streaming read / copy rate of one MI355X by buffer size (mpg_bw_probe):
where the Infinity Cache ends and how much of a small launch is fixed cost.

usage: python tools/probe_sizes.py [MB ...]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from __graft_entry__ import _load  # noqa: E402

m = _load()
sizes = [int(a) for a in sys.argv[1:]] or [4, 8, 16, 32, 64, 128, 192, 256, 512, 2048]
for mb in sizes:
    r = m.bw_probe("read", mb << 20, 5)
    c = m.bw_probe("copy", mb << 20, 5)
    print(f"{mb:6d} MB  read {r:8.0f} GB/s ({(mb << 20) / r / 1e3:8.2f} us)  copy {c:8.0f} GB/s", flush=True)
