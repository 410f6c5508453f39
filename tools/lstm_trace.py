"""Where the time of the persistent LSTM recurrences goes (csrc/lstm.hip lstm_fwd_pers /
lstm_bwd_pers, config-3 size): needs a library built with -DENCX_LSTM_TRACE, e.g.
  make -C encodec-pytorch_amd trace   (-> encodec-pytorch_amd/ab/trace.so)
  ENCX_LIB=encodec-pytorch_amd/ab/trace.so python tools/lstm_trace.py
Prints, per kernel and workgroup class, the median time of each phase of a frame and the
hand-off latency (a consumer's poll completing after the last producer's publish)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'encodec-pytorch_amd'))


def main():
    from encx._lib import call, ptr, lib
    B, H, T, L = (int(v) for v in os.environ.get('LSTM_SHAPE', '32,512,75,2').split(','))
    dev = torch.device('cuda', 0)
    g = torch.Generator(device='cpu').manual_seed(0)
    k = H ** -0.5
    f = lambda *s: ((torch.rand(*s, generator=g) * 2 - 1) * k).to(dev)
    e = lambda n: torch.empty(n, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    wcat, wcatT, bsum = e(L * 8 * H * H), e(L * 8 * H * H), e(L * 4 * H)
    for l in range(L):
        call('encx_lstm_pack', ptr(f(4 * H, H)), ptr(f(4 * H, H)), ptr(f(4 * H)), ptr(f(4 * H)), ptr(wcat), ptr(wcatT),
             ptr(bsum), H, l, st)
    x = torch.randn(B, H, T, generator=g).to(dev)
    dout = torch.randn(B, H, T, generator=g).to(dev)
    xt, Y, Cs, Gs, out = e(B * T * H), e(L * B * T * H), e(L * B * T * H), e(L * B * T * 4 * H), torch.empty_like(x)
    DA, dx = e(L * B * T * 4 * H), torch.empty_like(x)
    ws = torch.empty(lib.encx_lstm_bwd_workspace(B, T, H, L), dtype=torch.uint8, device=dev)
    for _ in range(3):
        call('encx_lstm_fwd', ptr(x), ptr(wcat), ptr(bsum), ptr(xt), ptr(Y), ptr(Cs), ptr(Gs), ptr(out), 1, B, T, H,
             L, st)
        call('encx_lstm_bwd', ptr(dout), ptr(wcatT), ptr(Cs), ptr(Gs), ptr(DA), ptr(dx), 0, ptr(ws), B, T, H, L, st)
    n = 2 * 256 * 128 * 8
    buf = np.zeros(n, dtype=np.int64)
    call('encx_lstm_trace', buf.ctypes.data_as(ctypes.c_void_p), n)
    tr = buf.reshape(2, 256, 128, 8).astype(np.float64) * 10.0 / 1000.0  # 100 MHz ticks -> us
    nbg = (B + 15) // 16
    # ---- forward: workgroup (l, bg, ug), NUG = H / 8
    nug = H // 8
    nwg = L * nbg * nug
    fw = tr[0, :nwg, :T]
    names = ['wait x', 'x MFMA', 'poll h', 'h load+MFMA+LDS', 'gates+stores', 'drain+barrier', 'to next frame']
    print(f'forward: {nwg} workgroups, frame cadence (median over workgroups of start(t+1) - start(t)): '
          f'{np.median(np.diff(fw[:, :, 0], axis=1)):.2f} us; whole recurrence '
          f'{fw[:, T - 1, 6].max() - fw[:, 0, 0].min():.1f} us')
    for l in range(L):
        sel = fw[l * nbg * nug:(l + 1) * nbg * nug, 1:]
        d = np.diff(np.concatenate([sel, np.roll(sel[:, :, :1], -1, axis=1)], axis=2), axis=2)[:, :-1]
        print(f'  layer {l}: ' + ', '.join(f'{nm} {np.median(d[:, :, i]):.2f}' for i, nm in enumerate(names)))
        # hand-off: poll h done (point 3) of frame t vs the last publish (point 6) of frame t-1 of the layer
        pub = sel[:, :, 6].max(axis=0)
        got = sel[:, 1:, 3]
        print(f'    h hand-off: last producer publish -> consumer poll done: median '
              f'{np.median(got - pub[None, :-1]):.2f} us, max {np.max(got - pub[None, :-1]):.2f}')
    # ---- backward: workgroup (l, bg, ct), NCT = 2H / 16
    nct = 2 * H // 16
    nwg = L * nbg * nct
    bw = tr[1, :nwg, :T]
    print(f'backward: {nwg} workgroups, frame cadence {np.median(np.diff(bw[:, :, 0], axis=1)):.2f} us; whole '
          f'recurrence {bw[:, T - 1, 5].max() - bw[:, 0, 0].min():.1f} us')
    nrt = H // 16
    for l in range(L):
        for kind, cts in (('recurrent', range(nrt, nct)), ('input', range(nrt))):
            ids = [(l * nbg + b) * nct + c for b in range(nbg) for c in cts]
            s = bw[ids][:, 1:]
            seg = lambda a, b: np.median(s[:, :, b] - s[:, :, a])
            print(f'  layer {l} {kind}: poll DA {seg(0, 1):.2f}, load+MFMA+LDS {seg(1, 2):.2f}, '
                  f'{"poll x " + format(seg(2, 3), ".2f") + ", " if kind == "recurrent" and l < L - 1 else ""}'
                  f'point phase {seg(3 if kind == "recurrent" and l < L - 1 else 2, 4):.2f}, drain+barrier {seg(4, 5):.2f}, '
                  f'to next frame {np.median(s[:, 1:, 0] - s[:, :-1, 5]):.2f}')
        rid = [(l * nbg + b) * nct + c for b in range(nbg) for c in range(nrt, nct)]
        pub = bw[rid][:, :, 5].max(axis=0)
        got = bw[rid][:, 1:, 1]
        print(f'    DA hand-off (recurrent tiles): last publish -> poll done: median '
              f'{np.median(got - pub[None, :-1]):.2f} us')


if __name__ == '__main__':
    main()
