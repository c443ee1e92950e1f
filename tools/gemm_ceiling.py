"""What does the vendor GEMM (hipBLASLt through torch.matmul, bf16) reach on the explicit-GEMM equivalents of the
C2 step's conv layers?  An implicit-GEMM conv cannot beat the explicit GEMM of the same M x N x K by much, so these
are realistic per-shape ceilings for the conv engine (not part of the product; torch is only the measuring stick).

    python tools/gemm_ceiling.py > gpurun_out/gemm_ceiling.txt
"""
import torch

# (name, M = pixels, N = output channels, K = Cin * k * k) at batch 16, 512x512 input
SHAPES = [
    ('384->128 k3 @128^2', 16 * 128 * 128, 128, 384 * 9),
    ('128->64 k3 @256^2', 16 * 256 * 256, 64, 128 * 9),
    ('64->64 k3 @256^2', 16 * 256 * 256, 64, 64 * 9),
    ('256->256 k3 @32^2', 16 * 32 * 32, 256, 256 * 9),
    ('128->128 k3 @64^2', 16 * 64 * 64, 128, 128 * 9),
    ('64->256 k1 @128^2', 16 * 128 * 128, 256, 64),
    ('256->1024 k1 @32^2', 16 * 32 * 32, 1024, 256),
    ('1024->256 k1 @32^2', 16 * 32 * 32, 256, 1024),
    ('512->512 k3 @16^2', 16 * 16 * 16, 512, 512 * 9),
    ('square 8192', 8192, 8192, 8192),
]


def timeit(fn, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device('cuda')
    for name, M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        bt = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: torch.matmul(a, b, out=out))
        us_t = timeit(lambda: torch.matmul(a, bt.t(), out=out))
        fl = 2.0 * M * N * K
        byt = 2.0 * (M * K + K * N + M * N)
        best = min(us, us_t)
        print(f'{name:22s} M {M:8d} N {N:5d} K {K:5d}: {us:8.1f} us (B [K][N]) {us_t:8.1f} us (B [N][K])  '
              f'{fl / best / 1e6:7.1f} TF/s  {byt / best / 1e3:6.2f} TB/s', flush=True)


if __name__ == '__main__':
    main()
