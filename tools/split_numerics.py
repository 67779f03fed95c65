import sys, numpy as np
sys.path.insert(0, '/root/repo/onitama-alphazero_amd'); sys.path.insert(0, '/root/repo/tests')
import oracle_ffi as orc
from onitama_az.weights import named_from_blob, random_weights
d = np.load('/root/repo/tests/golden/nn_golden.npz')
states = d['states']
planes = np.stack([orc.encode(s) for s in states]).astype(np.float64)  # [B,21,5,5]

def fold(t, conv, bn):
    w = t[f"{conv}|weight"].astype(np.float64); b = t[f"{conv}|bias"].astype(np.float64)
    s = t[f"{bn}|weight"].astype(np.float64) / np.sqrt(t[f"{bn}|running_var"].astype(np.float64) + 1e-5)
    wf = (w * s[:, None, None, None]).astype(np.float32)
    bf = ((b - t[f"{bn}|running_mean"]) * s + t[f"{bn}|bias"]).astype(np.float32)
    return wf, bf

def im2col(x):  # x [B,C,5,5] -> [B,25,C*9]
    B, C = x.shape[:2]
    xp = np.zeros((B, C, 7, 7), x.dtype); xp[:, :, 1:6, 1:6] = x
    cols = np.stack([xp[:, :, dy:dy + 5, dx:dx + 5] for dy in range(3) for dx in range(3)], -1)  # B C 5 5 9
    return cols.transpose(0, 2, 3, 1, 4).reshape(B, 25, C * 9)

def bf16_trunc(x):
    x = x.astype(np.float32); return (x.view(np.uint32) & 0xffff0000).view(np.float32)

def split_bf16x3(x):
    x = x.astype(np.float32); h = bf16_trunc(x); r = (x - h).astype(np.float32); m = bf16_trunc(r); l = (r - m).astype(np.float32)
    return h, m, l

def split_f16x2(x):
    x = x.astype(np.float32); h = x.astype(np.float16).astype(np.float32); l = (x - h).astype(np.float32).astype(np.float16).astype(np.float32)
    return h, l

def matmul(A, W, mode, wscale=None):
    # A [B,25,K] activations, W [Cout,K]
    if mode == 'f64': return A.astype(np.float64) @ W.astype(np.float64).T
    if mode == 'f32': return (A.astype(np.float32) @ W.astype(np.float32).T).astype(np.float64)
    if mode == 'x6':
        ah, am, al = split_bf16x3(A); wh, wm, wl = split_bf16x3(W)
        prods = [(ah, wh), (ah, wm), (am, wh), (ah, wl), (am, wm), (al, wh)]
    if mode == 'h3':
        s = wscale  # per-cout power of two
        ah, al = split_f16x2(A); wh, wl = split_f16x2(W * s[:, None])
        prods = [(ah, wh), (ah, wl), (al, wh)]
        return sum(a.astype(np.float64) @ w.astype(np.float64).T for a, w in prods) / s
    return sum(a.astype(np.float64) @ w.astype(np.float64).T for a, w in prods)

def forward(t, blocks, mode, stats=None):
    x = planes
    def conv(x, name, bn, relu=True, skip=None, first=False):
        wf, bf = fold(t, name, bn)
        W = wf.reshape(64, -1)
        s = 2.0 ** -np.floor(np.log2(np.abs(W).max(1) + 1e-30))
        y = matmul(im2col(x), W, 'f64' if first else mode, s) + bf  # [B,25,64]
        y = y.transpose(0, 2, 1).reshape(-1, 64, 5, 5)
        if skip is not None: y = y + skip
        y = np.maximum(y, 0) if relu else y
        if mode != 'f64': y = y.astype(np.float32).astype(np.float64)
        if stats is not None: stats.append((np.abs(y).max(), np.min(np.abs(y[y != 0])) if (y != 0).any() else 0))
        return y
    y = conv(x, 'conv_init_1', 'bn1', first=True)
    for i in range(blocks):
        p = f"resnet_{i}|resnet_small_block"
        y1 = conv(y, f"{p}1|small_block_conv", f"{p}1|small_block_bn")
        y = conv(y1, f"{p}2|small_block_conv", f"{p}2|small_block_bn", skip=y)
    B = y.shape[0]
    vw, vb = fold(t, 'vh_conv', 'vh_bn'); v = np.maximum(np.einsum('bchw,oc->bohw', y, vw.reshape(1, 64)) + vb[None, :, None, None], 0).reshape(B, -1)
    v = np.maximum(v @ t['vh_linear1|weight'].T.astype(np.float64) + t['vh_linear1|bias'], 0)
    v = np.tanh(v @ t['vh_linear2|weight'].T.astype(np.float64) + t['vh_linear2|bias']).reshape(-1)
    pw, pb = fold(t, 'policy_conv', 'policy_bn'); p = np.maximum(np.einsum('bchw,oc->bohw', y, pw.reshape(2, 64)) + pb[None, :, None, None], 0).reshape(B, -1)
    z = p @ t['ph_linear2|weight'].T.astype(np.float64) + t['ph_linear2|bias']
    z = np.exp(z - z.max(1, keepdims=True)); p = z / z.sum(1, keepdims=True)
    return p, v

for name, blob, blocks in (('trained3', np.load('/root/repo/tests/golden/weights_3block_trained.npy'), 3), ('random3', random_weights(0, 3), 3), ('random6', random_weights(1, 6), 6)):
    t = named_from_blob(blob, blocks)
    st = []
    p64, v64 = forward(t, blocks, 'f64', st)
    print(name, 'act range max %.3g minnz %.3g' % (max(a for a, b in st), min(b for a, b in st)))
    for mode in ('f32', 'x6', 'h3'):
        p, v = forward(t, blocks, mode)
        print('  %-4s dp %.3g dv %.3g' % (mode, np.abs(p - p64).max(), np.abs(v - v64).max()))

def rtz16(x):
    x = x.astype(np.float64)
    ax = np.abs(x); e = np.floor(np.log2(np.where(ax > 0, ax, 1.0)))
    q = 2.0 ** (np.maximum(e, -14) - 10)
    return (np.trunc(x / q) * q).astype(np.float32)
def split_rtz(x):
    x = x.astype(np.float32); h = rtz16(x); l = rtz16((x - h).astype(np.float32)); return h, l
split_f16x2 = split_rtz
print('--- RTZ split')
for name, blob, blocks in (('trained3', np.load('/root/repo/tests/golden/weights_3block_trained.npy'), 3), ('random6', random_weights(1, 6), 6)):
    t = named_from_blob(blob, blocks)
    p64, v64 = forward(t, blocks, 'f64')
    p, v = forward(t, blocks, 'h3')
    print('  %s h3rtz dp %.3g dv %.3g' % (name, np.abs(p - p64).max(), np.abs(v - v64).max()))
