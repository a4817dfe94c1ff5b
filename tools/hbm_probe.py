"""Calibrate the practical HBM rate on this GPU for the stream mixes the conv kernels see (torch copy /
add kernels on 2.95 GB fp32 tensors, the size of one C=48 x 240 000 x 64 activation):
1 read + 1 write (copy), 2 reads + 1 write (add), and 1 read + 2 writes (two copies of one source)."""
import torch


def timed(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    n = 48 * 240000 * 64
    a = torch.randn(n, device="cuda")
    b = torch.randn(n, device="cuda")
    c = torch.empty_like(a)
    d = torch.empty_like(a)
    gb = 4 * n / 1e9
    ms = timed(lambda: c.copy_(a))
    print(f"copy      1R+1W {2 * gb:6.2f} GB  {ms:7.3f} ms  {2 * gb / ms:6.2f} TB/s")
    ms = timed(lambda: torch.add(a, b, out=c))
    print(f"add       2R+1W {3 * gb:6.2f} GB  {ms:7.3f} ms  {3 * gb / ms:6.2f} TB/s")
    ms = timed(lambda: (c.copy_(a), d.copy_(a)))
    print(f"2 copies  2R+2W {4 * gb:6.2f} GB  {ms:7.3f} ms  {4 * gb / ms:6.2f} TB/s")
    ms = timed(lambda: a.sum())
    print(f"sum       1R    {gb:6.2f} GB  {ms:7.3f} ms  {gb / ms:6.2f} TB/s")
    ms = timed(lambda: c.fill_(1.0))
    print(f"fill      1W    {gb:6.2f} GB  {ms:7.3f} ms  {gb / ms:6.2f} TB/s")


if __name__ == "__main__":
    main()
