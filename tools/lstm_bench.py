"""LSTM recurrence timing (csrc/lstm.hip) at the config-3 size (B 32, H 512, T 75, L 2) under
kernel-selection option settings, each captured in a HIP graph and replayed (the form the training
step runs it in). Usage (GPU box): python tools/lstm_bench.py "LSTM_PERSIST=0" "LSTM_PERSIST=1" ...
Prints us per forward, backward and weight-grad pass (all layers) for every setting, and compares
every output and grad with the first setting's (bitwise, and the max difference)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'encodec-pytorch_amd'))


def main():
    from encx._lib import call, ptr, set_option, lib
    import ctypes
    B, H, T, L = (int(v) for v in os.environ.get('LSTM_SHAPE', '32,512,75,2').split(','))
    settings = sys.argv[1:] or ['-']
    dev = torch.device('cuda', 0)
    g = torch.Generator(device='cpu').manual_seed(0)
    k = H ** -0.5
    f = lambda *s: ((torch.rand(*s, generator=g) * 2 - 1) * k).to(dev)
    w = [(f(4 * H, H), f(4 * H, H), f(4 * H), f(4 * H)) for _ in range(L)]
    x = torch.randn(B, H, T, generator=g).to(dev)
    dout = torch.randn(B, H, T, generator=g).to(dev)
    e = lambda n: torch.empty(n, device=dev)
    wcat, wcatT, bsum = e(L * 8 * H * H), e(L * 8 * H * H), e(L * 4 * H)
    st = torch.cuda.current_stream().cuda_stream
    for l in range(L):
        call('encx_lstm_pack', *(ptr(t) for t in w[l]), ptr(wcat), ptr(wcatT), ptr(bsum), H, l, st)
    xt, Y, Cs, Gs, out = e(B * T * H), e(L * B * T * H), e(L * B * T * H), e(L * B * T * 4 * H), torch.empty_like(x)
    DA, dx = e(L * B * T * 4 * H), torch.empty_like(x)
    ws = torch.empty(lib.encx_lstm_bwd_workspace(B, T, H, L), dtype=torch.uint8, device=dev)

    def fwd():
        call('encx_lstm_fwd', ptr(x), ptr(wcat), ptr(bsum), ptr(xt), ptr(Y), ptr(Cs), ptr(Gs), ptr(out), 1, B, T, H, L,
             torch.cuda.current_stream().cuda_stream)

    def bwd():
        call('encx_lstm_bwd', ptr(dout), ptr(wcatT), ptr(Cs), ptr(Gs), ptr(DA), ptr(dx), 0, ptr(ws), B, T, H, L,
             torch.cuda.current_stream().cuda_stream)

    dws = [[torch.empty(4 * H, H, device=dev), torch.empty(4 * H, H, device=dev), torch.empty(4 * H, device=dev),
            torch.empty(4 * H, device=dev)] for _ in range(L)]

    def wgrad():
        wsw = torch.empty(lib.encx_lstm_bwd_weight_workspace(B, T, H), dtype=torch.uint8, device=dev)
        for l in range(L):
            call('encx_lstm_bwd_weight', ptr(DA), ptr(xt), ptr(Y), *(ptr(t) for t in dws[l]), 0, ptr(wsw), B, T, H, L,
                 l, torch.cuda.current_stream().cuda_stream)

    def timed(fn, reps=20):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    ref = None
    for sset in settings:
        kv = [] if sset == '-' else [p.split('=') for p in sset.split(',')]
        prev = {kk: set_option(kk, int(v)) for kk, v in kv}
        tf = timed(fwd)
        tb = timed(bwd)
        fwd()
        bwd()
        tw = timed(wgrad)
        wgrad()
        torch.cuda.synchronize()
        n = ctypes.c_int64()
        call('encx_lstm_sync_errors', ctypes.byref(n))
        got = [t.clone() for t in (out, Y, Cs, Gs, DA, dx, *[w for d in dws for w in d])]
        if ref is None:
            ref = got
        diff = max(float((a - b).abs().max()) for a, b in zip(got, ref))
        same = all(torch.equal(a, b) for a, b in zip(got, ref))
        print(f'{sset}: fwd {tf:.1f} us, bwd {tb:.1f} us, weight grads {tw:.1f} us; vs first setting: bitwise {same}, max diff {diff:.3g}; '
              f'sync errors {n.value}', flush=True)
        for kk, v in prev.items():
            set_option(kk, v)


if __name__ == '__main__':
    main()
