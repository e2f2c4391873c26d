"""Every size-matched probe shape (tools/bench_loop.hip stream_rw_kernel family) on a few byte
shapes: the headline (config 2), the 16M shard and the two tx_build lines. Tools only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def main():
    import torch

    dev = torch.device("cuda:0")
    d = bench.Dist()
    n = 1 << 20
    shapes = [("config2", n * 70, n * 32, 16), ("config4_shard_16M", 16 * n * 70, 16 * n * 32, 2),
              ("tx_build_64B", n * 62, n * 67, 1), ("tx_build_1514B", (n // 4) * 1512, (n // 4) * 1519, 1)]
    for name, rb, wb, nbuf in shapes:
        k = bench.size_matched_probe(dev, rb, wb, d, nbuf=nbuf)
        print(name, f"best {k:.5f} ms", bench.LAST_PROBE_SHAPES, flush=True)


if __name__ == "__main__":
    main()
