"""TOOLS ONLY: give round 4's facade_check (extracted from git by the Makefile) today's `time` mode, which also times
the reader's and the RawPacket's destruction, so tools/facade_probe.py compares the same phases for both facades.

  python port_time_mode.py <round-4 facade_check.cpp> <today's tests/native/facade_check.cpp>   (rewrites the first)
"""
import sys
from pathlib import Path


def time_mode(src: str) -> str:
    a = src.index("int timeMode(const char* capture, int reps)")
    return src[a:src.index("}  // namespace", a)]


old, new = Path(sys.argv[1]), Path(sys.argv[2])
s = old.read_text()
s = s.replace(time_mode(s), time_mode(new.read_text()))
old.write_text(s)
