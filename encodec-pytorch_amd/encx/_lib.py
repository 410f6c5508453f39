"""ctypes binding of libencx.so (the C ABI declared in include/encx.h).

The signatures are read from the header itself, so the binding can never drift from the
declared boundary. There is no fallback: if the HIP library is missing or fails to load, every
encx op raises. Tensors cross the boundary as raw device pointers + sizes, on torch's current
HIP stream.
"""
import ctypes
import os
import re

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('ENCX_LIB', os.path.join(_HERE, 'libencx.so'))
HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), 'include', 'encx.h')

_CTYPES = {
    'int': ctypes.c_int, 'int64_t': ctypes.c_int64, 'uint64_t': ctypes.c_uint64,
    'size_t': ctypes.c_size_t, 'float': ctypes.c_float, 'double': ctypes.c_double,
    'encx_stream_t': ctypes.c_void_p, 'const char*': ctypes.c_char_p,
}

ENCX_PAD_ZERO, ENCX_PAD_REFLECT = 0, 1
ENCX_ACT_NONE, ENCX_ACT_ELU = 0, 1
ENCX_AC_STATE, ENCX_AC_MAXBIT, ENCX_AC_POS = 8, 6, 7  # arithmetic-decoder state words (encx.h)
ENCX_BALANCER_MAX_LOSSES = 64  # encx.h


def _ctype(t):
    t = ' '.join(t.replace('*', ' * ').split()).replace(' *', '*')
    if t in _CTYPES:
        return _CTYPES[t]
    if t.endswith('*'):
        return ctypes.c_void_p
    if t == 'void':
        return None
    raise TypeError(f'unmapped C type {t!r}')


def parse_header(path=HEADER):
    """-> {name: (restype, [argtypes])} for every encx_* function declared in the header."""
    src = open(path).read()
    src = re.sub(r'/\*.*?\*/', ' ', src, flags=re.S)
    src = re.sub(r'//[^\n]*', ' ', src)
    src = re.sub(r'^\s*#.*$', ' ', src, flags=re.M)
    out = {}
    for stmt in src.split(';'):
        stmt = re.split(r'[{}]', stmt)[-1].strip()
        m = re.match(r'^([\w\s\*]+?)\b(encx_\w+)\s*\(([^)]*)\)$', stmt, re.S)
        if not m or stmt.startswith('typedef'):
            continue
        ret, name, args = ' '.join(m.group(1).split()), m.group(2), m.group(3).strip()
        argtypes = []
        if args and args != 'void':
            for a in args.split(','):
                a = ' '.join(a.split())
                am = re.match(r'(.*?)(\w+)$', a)
                argtypes.append(_ctype(am.group(1).strip()))
        out[name] = (_ctype(ret), argtypes)
    return out


def check_build_id(lib):
    """Refuse a library built from other sources than the ones beside it (buildid.py). An A/B
    build picked with ENCX_LIB is an experiment: a mismatch there only warns."""
    import sys
    sys.path.insert(0, os.path.dirname(_HERE))
    try:
        from buildid import build_id
    finally:
        sys.path.pop(0)
    want, have = build_id(), lib.encx_build_id().decode()
    if want == have:
        return
    msg = (f'encx: {LIB_PATH} was built from other sources (build id {have}, sources {want}); '
           'rebuild with `make -C encodec-pytorch_amd`')
    if 'ENCX_LIB' in os.environ:
        print('warning: ' + msg, file=sys.stderr)
        return
    raise RuntimeError(msg)


class _Lib:
    def __init__(self):
        self._lib = None
        self.sigs = parse_header()

    def load(self):
        if self._lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f'encx: HIP library not built ({LIB_PATH}); run '
                                   '`python -c "import __graft_entry__ as g; g.build()"` '
                                   'or `make -C encodec-pytorch_amd`')
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in self.sigs.items():
                if 'ENCX_LIB' in os.environ and not hasattr(lib, name):
                    continue  # an A/B build of an older revision: entry points added since are absent
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            check_build_id(lib)
            self._lib = lib
        return self._lib

    def __getattr__(self, name):
        if not name.startswith('encx_'):
            raise AttributeError(name)
        return getattr(self.load(), name)


lib = _Lib()


def check(rc, what=''):
    if rc != 0:
        msg = lib.encx_strerror(rc)
        raise RuntimeError(f'encx {what} failed: {msg.decode() if msg else rc} (code {rc})')


def call(name, *args):
    check(getattr(lib, name)(*args), name)


def get_option(name):
    v = ctypes.c_int64()
    call('encx_get_option', name.encode(), ctypes.byref(v))
    return v.value


def set_option(name, value):
    """Set a kernel-selection option (encx.h encx_set_option); returns the previous value."""
    prev = ctypes.c_int64()
    call('encx_set_option', name.encode(), int(value), ctypes.byref(prev))
    return prev.value


def options():
    """{name: current value} of every kernel-selection option."""
    names = [lib.encx_option_name(i).decode() for i in range(lib.encx_option_count())]
    return {n: get_option(n) for n in names}


class option:
    """`with option(DGR=256, ...):` -- set options for a block, restore them after."""

    def __init__(self, **kv):
        self.kv = kv
        self.prev = {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.prev[k] = set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.prev.items():
            set_option(k, v)
        return False


def lstm_sync_errors():
    """Hand-off spins of the persistent LSTM kernels that timed out since the last call (encx.h
    encx_lstm_sync_errors; synchronises the device)."""
    n = ctypes.c_int64()
    call('encx_lstm_sync_errors', ctypes.byref(n))
    return n.value


def ptr(t):
    """Device pointer of a contiguous fp32/int64 CUDA tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError('encx ops take device tensors (no CPU fallback)')
    if not t.is_contiguous():
        raise RuntimeError('encx ops take contiguous tensors')
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


_inited = set()


def ensure_device(dev):
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _inited:
        call('encx_init', idx)
        _inited.add(idx)
