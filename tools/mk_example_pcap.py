"""Writes the reference example.pcap (frozen in tests/golden/capture_example.npz) to the path given (GPU-box profiling runs)."""
import sys
from pathlib import Path
R = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(R)); sys.path.insert(0, str(R / 'tests'))
from conftest import GOLDEN, load_golden
from pcapplusplus_amd.pcap import write_pcap
ex, _ = load_golden(GOLDEN / "capture_example.npz")
write_pcap(sys.argv[1], ex)
print(ex.n)
