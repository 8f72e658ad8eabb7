"""Host helpers to read the engine's tiled HBM layout back (include/ocx.h)."""
import numpy as np


def untile_z(zt: np.ndarray, L) -> np.ndarray:
    """z_tiled (flat, G*T*64*C) → z [B, T, d]."""
    G, T, C, P, S = L.G, L.T, L.C, L.P, L.S
    a = zt.reshape(G, T, C // 2, 64, 2)            # [g][t][k][lane][e]
    a = a.reshape(G, T, C // 2, S, P, 2)            # lane = s*P + c
    a = a.transpose(0, 3, 1, 4, 2, 5)               # [g][s][t][c][k][e]
    a = a.reshape(G * S, T, P * C)                  # j = c*C + 2k + e
    return a[:L.B, :, :L.d]


def untile_y(yt: np.ndarray, L) -> np.ndarray:
    a = yt.reshape(L.G, L.T, L.S).transpose(0, 2, 1).reshape(L.G * L.S, L.T)
    return a[:L.B]
