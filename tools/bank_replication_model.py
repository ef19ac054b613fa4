"""Bank-conflict model (tools/bank_model.py) of the C2 tile kernel with the hot
table replicated 2/4/8 times at rotated offsets, the copy chosen by lane: extra
LDS cycles per lookup wave-instruction (modeled, dropped:
replication breaks the same-dword broadcast of lanes in one state)."""
import sys, numpy as np
import os; _R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, os.path.join(_R, 'tools')); sys.path.insert(0, _R)
from bank_model import lane_states
states, hay, hot = lane_states(waves=24)
L, N = states.shape
pitch = 304
def conf(ncopies, cstride):
    lane = np.arange(N) % 64
    base = (lane % ncopies) * cstride
    addr = base[None, :] + states * pitch + hay.T.astype(np.int64)
    dw = addr >> 2; bank = dw & 31
    total = 0; count = 0
    for g0 in range(0, N, 32):
        d = dw[:, g0:g0+32]; b = bank[:, g0:g0+32]
        key = b * (1 << 40) + d
        ks = np.sort(key, axis=1)
        uniq = np.concatenate([np.ones((L,1),bool), ks[:,1:] != ks[:,:-1]], axis=1)
        bk = ks >> 40
        per = np.zeros((L, 32), dtype=np.int64)
        rows = np.repeat(np.arange(L), 32)
        np.add.at(per, (rows, bk.ravel()), uniq.ravel().astype(np.int64))
        total += (per.max(axis=1) - 1).sum(); count += L
    return total / (count / 2)
rows_bytes = (hot + 1) * pitch
print('1 copy', conf(1, 0))
for n in (2, 4, 8):
    for extra in (0, 4, 8, 16, 64):
        print(n, 'copies stride', rows_bytes + extra, round(conf(n, rows_bytes + extra), 3))
