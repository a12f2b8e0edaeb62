"""Model of the cross-XCD operand re-reads of the B = 20 combined launch
(tcu_kernel: job I' + the fused update), the part of its PMC fetch above the
algorithmic bytes that the tile placement implies.  Each XCD has its own L2,
so an operand slice read by tiles on k XCDs is fetched k times from beyond L2
(MALL / HBM), while bench.kernel_work("tcu") counts it once.
  - update tiles: 64 x 64 tiles of W_aug, tile index tm-fastest inside a layer,
    consecutive index ranges per XCD (upd_body in csrc/iwae_update_dev.h: the
    sample-row tiles spread over the 8 XCDs first, the image-row tiles after);
    a tile reads its X slice (rows x 64 inputs) and its dZ slice (rows x 64 outputs);
  - job I': 20 image workgroups on blockIdx & 7, each streaming the GX copies of
    e1.l2 and e1.head (hi + lo bf16, 4 B per weight).
    python tools/xcd_reread_model.py [sample_rows] [images]"""
import sys


def cd(a, b):
    return -(-a // b)


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    img = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    jobs = [("e2.l1", 100, 100, S), ("e2.l2", 100, 100, S), ("e2.head", 100, 100, S), ("p.l1", 50, 100, S),
            ("p.l2", 100, 100, S), ("p.head", 100, 200, S), ("o.l1", 100, 200, S), ("o.l2", 200, 200, S),
            ("o.l3", 200, 784, S), ("e1.l1", 784, 200, img), ("e1.l2", 200, 200, img), ("e1.head", 200, 200, img)]
    tiles = []
    for n, fi, fo, r in jobs:
        tm, tn = cd(fi + 1, 64), cd(fo, 64)
        for lt in range(tm * tn):
            b, a = divmod(lt, tm)
            tiles.append((n, fi, fo, r, a, b))
    heavy = sum(1 for t in tiles if t[3] == S)
    per, per2 = cd(heavy, 8), cd(len(tiles) - heavy, 8)
    once, per_x = {}, [dict() for _ in range(8)]
    for T, (n, fi, fo, r, a, b) in enumerate(tiles):
        x = T // per if T < heavy else (T - heavy) // per2
        for key, by in (((n, "X", a), r * min(64, fi + 1 - 64 * a) * 4), ((n, "Z", b), r * min(64, fo - 64 * b) * 4)):
            per_x[x][key] = by
            once[key] = by
    alg = sum(once.values())
    dup = sum(sum(s.values()) for s in per_x)
    wI = 4 * (200 * 200 + 200 * 200)
    nx = min(8, img)
    print(f"update X / dZ slices: once {alg / 1e6:.2f} MB, summed over the XCDs' L2s {dup / 1e6:.2f} MB "
          f"(+{(dup - alg) / 1e6:.2f} MB)")
    print(f"job I' weights (e1.l2^T, e1.head^T GX copies): once {wI / 1e6:.2f} MB, on {nx} XCDs {nx * wI / 1e6:.2f} MB "
          f"(+{(nx - 1) * wI / 1e6:.2f} MB)")
    print(f"modeled re-read total: +{(dup - alg + (nx - 1) * wI) / 1e6:.2f} MB per launch")


if __name__ == "__main__":
    main()
