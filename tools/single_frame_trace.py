"""The drop-in per-callback path alone (bench.py's single_frame block: 1M-point pageable
host clouds -> c3h_voxelize -> c3h_extract -> c3h_search, one frame at a time), for a
kernel / memory-copy trace: rocprofv3 --kernel-trace --memory-copy-trace --stats -- python3
tools/single_frame_trace.py [frames].  Prints the block as one JSON line."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "mapping-private_amd")]


def main():
    import torch
    import bench
    import c3hlac
    from c3hlac import synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    torch.cuda.init()
    print(json.dumps(bench.single_frame_pass(0, torch, synth, c3hlac, 0, n)))


if __name__ == "__main__":
    main()
