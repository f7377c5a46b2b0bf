"""fp32 error of Winograd F(2x2,3x3) and F(4x4,3x3) (two point sets)
against a float64 direct conv, beside the direct fp32 conv, on the four
channel shapes of blocks 1-4 (random ReLU activations, Glorot weights).
Every operand / product / sum in fp32 as the kernels compute; U from float64
rounded once.  Output: profiles/r04_wino_f43_error.txt."""
import numpy as np, sympy as sp, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
from mats import winograd_mats

def f64(M): return np.array([[float(x) for x in M.row(i)] for i in range(M.rows)])

def direct64(x, w):  # x [T][F][Cin] , w [Cout][Cin][3][3]
    T, F, C = x.shape
    xp = np.zeros((T + 2, F + 2, C)); xp[1:-1, 1:-1] = x
    out = np.zeros((T, F, w.shape[0]))
    for dy in range(3):
        for dx in range(3):
            out += xp[dy:dy + T, dx:dx + F] @ w[:, :, dy, dx].T
    return out

def direct32(x, w):
    T, F, C = x.shape
    xp = np.zeros((T + 2, F + 2, C), np.float32); xp[1:-1, 1:-1] = x
    out = np.zeros((T, F, w.shape[0]), np.float32)
    w32 = w.astype(np.float32)
    for c in range(C):                     # K order: channel outer, tap inner (sequential fp32)
        for dy in range(3):
            for dx in range(3):
                out = out + xp[dy:dy + T, dx:dx + F, c:c + 1] * w32[None, None, :, c, dy, dx]
    return out

def wino32(x, w, m, pts):
    AT, G, BT = winograd_mats(pts, m, 3)
    AT, G, BT = f64(AT), f64(G), f64(BT)
    n = m + 2
    T, F, C = x.shape
    Co = w.shape[0]
    U = np.einsum('ik,ockl,jl->ijoc', G, w, G).astype(np.float32)   # [n][n][Co][C], float64 then rounded
    To, Fo = -(-T // m), -(-F // m)
    xp = np.zeros((To * m + 2, Fo * m + 2, C), np.float32); xp[1:T + 1, 1:F + 1] = x
    # patches [To][Fo][n][n][C]
    P = np.stack([np.stack([xp[a * m:a * m + n, b * m:b * m + n] for b in range(Fo)]) for a in range(To)])
    BT32, AT32 = BT.astype(np.float32), AT.astype(np.float32)
    # V = BT d B in fp32 (rows then columns)
    V = np.einsum('ir,abrcC->abicC', BT32, P).astype(np.float32)
    V = np.einsum('abirC,jr->abijC', V, BT32).astype(np.float32)      # [To][Fo][n][n][C]
    M = np.zeros((To, Fo, n, n, Co), np.float32)
    for c in range(C):
        M = M + V[..., c:c + 1] * U[None, None, :, :, :, c]
    Y = np.einsum('ir,abrsO->abisO', AT32, M).astype(np.float32)
    Y = np.einsum('abisO,js->abijO', Y, AT32).astype(np.float32)     # [To][Fo][m][m][Co]
    Y = Y.transpose(0, 2, 1, 3, 4).reshape(To * m, Fo * m, Co)
    return Y[:T, :F]

rng = np.random.default_rng(0)
for (T, F, C, Co) in ((50, 32, 64, 64), (50, 32, 128, 128), (40, 16, 256, 256), (40, 8, 512, 512)):
    x = np.maximum(rng.normal(0, 1, (T, F, C)), 0).astype(np.float32)
    w = (rng.uniform(-1, 1, (Co, C, 3, 3)) * np.sqrt(6.0 / (9 * C + 9 * Co))).astype(np.float64)
    ref = direct64(x.astype(np.float64), w)
    rms = np.sqrt(np.mean(ref ** 2))
    res = {'direct32': direct32(x, w), 'F2': wino32(x, w, 2, [0, 1, -1]),
           'F4(+-2)': wino32(x, w, 4, [0, 1, -1, 2, -2]),
           'F4(+-1/2)': wino32(x, w, 4, [0, 1, -1, sp.Rational(1, 2), -sp.Rational(1, 2)])}
    print('T%d F%d %d->%d  rms %.3g' % (T, F, C, Co, rms),
          '  '.join('%s max %.2e rms %.2e' % (k, np.max(np.abs(v - ref)), np.sqrt(np.mean((v - ref) ** 2))) for k, v in res.items()))
