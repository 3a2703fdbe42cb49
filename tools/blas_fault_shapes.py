"""Host-side arithmetic of the round-4 library-GEMM fault (NIDT_R3D_BLAS=1 at config-5 scale, profiles/r4_blas_1x1_fault.txt):
the batched torch.bmm operands of every 1x1x1 stride-1 conv of the 3D ResNet-50 at 32 clients x 4 volumes, with
their element counts, byte sizes and batch strides against 2^31.  Nothing runs on a GPU.
Usage: python tools/blas_fault_shapes.py"""

LIM = 2 ** 31


def main():
    G, B = 32, 4
    # (layer, spatial positions per volume, [(cin, cout)] of the stride-1 1x1x1 convs incl. their data gradients)
    stages = [("layer1", 31 * 37 * 31, [(64, 64), (64, 256), (256, 64)]),
              ("layer2", 16 * 19 * 16, [(128, 512), (512, 128)]),
              ("layer2.0.conv1", 31 * 37 * 31, [(256, 128)]),
              ("layer3", 8 * 10 * 8, [(256, 1024), (1024, 256)]),
              ("layer3.0.conv1", 16 * 19 * 16, [(512, 256)]),
              ("layer4", 4 * 5 * 4, [(512, 2048), (2048, 512)]),
              ("layer4.0.conv1", 8 * 10 * 8, [(1024, 512)])]
    print("%-16s %6s %6s %12s %14s %14s %12s %s" % ("stage", "K", "N", "rows/client", "X elems", "Y elems", "max bytes",
                                                   "exceeds 2^31"))
    worst_e = worst_b = 0
    for name, S, convs in stages:
        Mg = B * S
        for K, N in convs:
            for k, n in ((K, N), (N, K)):  # forward and data gradient
                xe, ye = G * Mg * k, G * Mg * n
                mb = 2 * max(xe, ye)
                worst_e, worst_b = max(worst_e, xe, ye), max(worst_b, mb)
                flags = []
                if max(xe, ye) >= LIM:
                    flags.append("ELEMENTS")
                if mb >= LIM:
                    flags.append("bytes")
                if Mg * max(k, n) >= LIM:
                    flags.append("batch stride")
                print("%-16s %6d %6d %12d %14d %14d %12d %s" % (name, k, n, Mg, xe, ye, mb, ",".join(flags) or "-"))
    print("largest operand: %d elements (%.3f x 2^31), %d bytes (%.3f x 2^31)" % (worst_e, worst_e / LIM, worst_b,
                                                                                 worst_b / LIM))


if __name__ == "__main__":
    main()
