"""Host helpers to read the engine's tiled HBM layout back (include/ocx.h)."""
import numpy as np


def untile_z(zt: np.ndarray, L) -> np.ndarray:
    """z_tiled (flat, (C/2)*G*T*128) → z [B, T, d]."""
    G, T, C, P, S = L.G, L.T, L.C, L.P, L.S
    a = zt.reshape(C // 2, G, T, S, P, 2)      # [k][g][t][s][c][e], lane = s*P + c
    a = a.transpose(1, 3, 2, 4, 0, 5)           # [g][s][t][c][k][e]
    a = a.reshape(G * S, T, P * C)              # j = c*C + 2k + e
    return a[:L.B, :, :L.d]


def untile_y(yt: np.ndarray, L) -> np.ndarray:
    a = yt.reshape(L.G, L.T, L.S).transpose(0, 2, 1).reshape(L.G * L.S, L.T)
    return a[:L.B]
