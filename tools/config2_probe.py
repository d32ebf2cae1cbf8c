"""bench.py's config #2 line alone (GPU box): python tools/config2_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    for _ in range(2):
        print(json.dumps(bench.config2_line(dev)), flush=True)


if __name__ == "__main__":
    main()
