"""Model of the LDS bank conflicts of the tile kernel's DFA lookups
(diagnostic, not part of the library).

Each ds_read_u8 of a wave is serviced as two 32-lane groups; within a group
lanes reading different dwords on one bank ((addr / 4) mod 32) serialise
(MI355X_MICROARCH.md §LDS).  The lookup address is row(s) * pitch + byte.
This walks C2-like haystacks through the exported forward DFA exactly as the
tile kernel does (hot rows, absorbing sentinel) and reports the mean extra
cycles per lookup for a row pitch and a row order, so layouts can be compared
on the CPU; the GPU counter (SQ_LDS_BANK_CONFLICT) checks the model.

  python tools/bank_model.py [pitch ...]
"""
import itertools
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import regex_amd as R  # noqa: E402
from regex_amd.workloads import date_haystacks_host  # noqa: E402


def lane_states(pat=r"\d{4}-\d{2}-\d{2}", waves=48, L=1024, seed=7):
    info, trans, eof, start = R.Regex(pat).dfa_tables(0)
    hot = int(R.Regex(pat).dfa_info(0)["normal"])
    hot = min(hot, 15)
    buf, _ = date_haystacks_host(waves * 64, L, seed=seed)
    hay = buf.reshape(waves * 64, L)
    s0 = int(start[1 | 4 | 32])  # start of text and of a line, no word byte before or after
    s = np.full(waves * 64, s0 if s0 < hot else hot, dtype=np.int64)
    states = np.empty((L, waves * 64), dtype=np.int64)
    for i in range(L):
        states[i] = s
        nxt = trans[np.minimum(s, trans.shape[0] - 1), hay[:, i]].astype(np.int64)
        s = np.where((s < hot) & (nxt < hot), nxt, hot)
    return states, hay, hot


def conflicts(states, hay, row_of, pitch):
    """Mean extra LDS cycles per wave-level lookup."""
    L, N = states.shape
    addr = row_of[states] * pitch + hay.T.astype(np.int64)
    dw = addr >> 2
    bank = dw & 31
    total = 0
    count = 0
    for g0 in range(0, N, 32):
        d = dw[:, g0:g0 + 32]
        b = bank[:, g0:g0 + 32]
        # distinct dwords per bank, max over banks, per step
        key = b * (1 << 40) + d
        ks = np.sort(key, axis=1)
        uniq = np.concatenate([np.ones((L, 1), bool), ks[:, 1:] != ks[:, :-1]], axis=1)
        bk = ks >> 40
        per_bank = np.zeros((L, 32), dtype=np.int64)
        rows = np.repeat(np.arange(L), 32)
        np.add.at(per_bank, (rows, bk.ravel()), uniq.ravel().astype(np.int64))
        total += (per_bank.max(axis=1) - 1).sum()
        count += L
    return total / (count / 2)   # per wave instruction (two groups)


def main():
    states, hay, hot = lane_states()
    occ = np.bincount(states.ravel(), minlength=hot + 1) / states.size
    print("hot", hot, "state occupancy", np.round(occ, 3))
    ident = np.arange(hot + 1)
    pitches = [int(x) for x in sys.argv[1:]] or [256, 272, 288, 304, 320, 336, 352, 368, 384, 400]
    for p in pitches:
        print("pitch %d: %.3f extra cycles per lookup" % (p, conflicts(states, hay, ident, p)))


if __name__ == "__main__":
    main()
