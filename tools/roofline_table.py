"""Algorithmic roofline of every ResNet152 conv class at the bench shape (B=128, bf16 NHWC).

FLOPs = 2*M*N*K (real Cin for the stem).  Bytes = input activation read once (not the im2col
expansion) + weights + output + residual (c3 / downsample-fed adds), all bf16.  Bound = the larger
of FLOPs / 2.5 PFLOP/s (dense bf16 MFMA) and bytes / 6.3 TB/s (achievable HBM3E,
MI355X_MICROARCH.md §HBM).  Prints a markdown table.
"""
B = 128
PEAK_TF, HBM_TBS = 2500.0, 6.3


def convs():
    out = [("stem 7x7/2", B * 112 * 112, 64, 7 * 7 * 3, B * 224 * 224 * 8, 0)]
    h, cin = 56, 64
    for li, (n, pl) in enumerate(zip([3, 8, 36, 3], [64, 128, 256, 512])):
        for bi in range(n):
            s = (1 if li == 0 else 2) if bi == 0 else 1
            oh = h // s
            out.append((f"L{li + 1} c1 1x1", B * h * h, pl, cin, B * h * h * cin, 0))
            out.append((f"L{li + 1} c2 3x3", B * oh * oh, pl, 9 * pl, B * h * h * pl, 0))
            if bi == 0:
                out.append((f"L{li + 1} ds 1x1", B * oh * oh, 4 * pl, cin, B * h * h * cin, 0))
            out.append((f"L{li + 1} c3 1x1+res", B * oh * oh, 4 * pl, pl, B * oh * oh * pl, 1))
            cin, h = 4 * pl, oh
    return out


def main():
    agg = {}
    for name, M, N, K, in_elems, res in convs():
        a = agg.setdefault((name, M, N, K), [0, 0.0, 0.0, (M, N, K)])
        a[0] += 1
        a[1] += 2.0 * M * N * K
        a[2] += 2.0 * (in_elems + N * K + M * N * (2 if res else 1))
    print("| conv class | n | M x N x K | GFLOP/launch | MB/launch | FLOP/B | bound | floor µs (all launches) |")
    print("|---|---|---|---|---|---|---|---|")
    tot_f = tot_t = 0.0
    for (name, _, _, _), (n, f, by, (M, N, K)) in agg.items():
        t_m = f / (PEAK_TF * 1e12) * 1e6
        t_h = by / (HBM_TBS * 1e12) * 1e6
        tot_f += f
        tot_t += max(t_m, t_h)
        print(f"| {name} | {n} | {M}x{N}x{K} | {f / n / 1e9:.2f} | {by / n / 1e6:.1f} | {f / by:.0f} | "
              f"{'MFMA' if t_m > t_h else 'HBM'} | {max(t_m, t_h):.0f} |")
    print(f"\ntotal {tot_f / 1e12:.3f} TFLOP per forward; roofline floor {tot_t:.0f} µs")


if __name__ == "__main__":
    main()
