"""Graph replay vs eager trainer, bitwise, per step (tests/test_gpu_train_state.py's two-key
case), printing the first mismatch per step and the persistent LSTM's hand-off timeouts.
Usage (GPU box): ENCX_LSTM_PERSIST=0|1 python tools/diag/graph_vs_eager.py"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
sys.path.insert(0, os.path.join(ROOT, 'encodec-pytorch_amd'))
sys.path.insert(0, ROOT)
from test_gpu_train_state import make_trainer, batches  # noqa: E402
from encx._lib import call  # noqa: E402


def errs():
    n = ctypes.c_int64()
    call('encx_lstm_sync_errors', ctypes.byref(n))
    return n.value


def main():
    xs = batches(6)
    runs = []
    for graphs in (False, True):
        tr = make_trainer(graphs=graphs)
        per = []
        for i, x in enumerate(xs):
            tr.model.target_bandwidths = [6.0 if i % 2 == 0 else 3.0]
            tr.step(x)
            torch.cuda.synchronize()
            per.append([t.clone() for t in (tr.opt.flat_grad, tr.opt.flat, tr.opt_d.flat_grad, tr.opt_d.flat)])
            print(f'graphs={graphs} step {i}: lstm sync errors {errs()}', flush=True)
        runs.append(per)
    for i, (a, b) in enumerate(zip(*runs)):
        d = [float((ta - tb).abs().max()) for ta, tb in zip(a, b)]
        print(f'step {i}: max |eager - graph| gen_grad {d[0]:.3g} gen {d[1]:.3g} disc_grad {d[2]:.3g} disc {d[3]:.3g}',
              flush=True)


if __name__ == '__main__':
    main()
