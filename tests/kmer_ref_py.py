"""Pure-Python statement of the reference's k-mer semantics,
written over strings with no bit tricks, for small independent cross-checks of
the C oracle. TEST INFRASTRUCTURE.

key(read, p): the 32*W bases starting at p, where bases past the read end read
as 'A' (code 0) and any byte outside ACGT reads as 'T' (code 3); when
ceil(k/4) < 8*W the bases from k on are cleared to 'A' (GPUHandler.cu:181-186).
A window is counted when s[p:p+k] is all ACGT; if any window is not, the key
0^W is present with (at least) count 0.
"""
from collections import Counter

CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def key_of(s: str, p: int, k: int):
    W = (k + 31) // 32
    mask = ((k + 3) // 4) < 8 * W
    t = []
    for i in range(32 * W):
        j = p + i
        if mask and i >= k:
            c = "A"
        elif j >= len(s):
            c = "A"
        else:
            c = s[j] if s[j] in CODE else "T"
        t.append(c)
    words = []
    for w in range(W):
        v = 0
        for c in t[32 * w:32 * w + 32]:
            v = (v << 2) | CODE[c]
        words.append(v)
    return tuple(words)


def count_reads(reads, k: int) -> Counter:
    cnt = Counter()
    hole = False
    for s in reads:
        for p in range(len(s) - k + 1):
            if all(ch in CODE for ch in s[p:p + k]):
                cnt[key_of(s, p, k)] += 1
            else:
                hole = True
    if hole:
        cnt[tuple([0] * ((k + 31) // 32))] += 0
    return cnt


def to_bytes(cnt: Counter, k: int) -> bytes:
    W = (k + 31) // 32
    out = bytearray()
    for key in sorted(cnt):
        for w in key:
            out += int(w).to_bytes(8, "little")
        out += (cnt[key] & 0xFFFFFFFF).to_bytes(4, "little")
    return bytes(out)


def parse_records(data: bytes, k: int):
    W = (k + 31) // 32
    rs = 8 * W + 4
    out = []
    for i in range(0, len(data) - len(data) % rs, rs):
        key = tuple(int.from_bytes(data[i + 8 * j:i + 8 * j + 8], "little") for j in range(W))
        out.append((key, int.from_bytes(data[i + 8 * W:i + rs], "little")))
    return out


def fastq_reads(text: str):
    """Sequence lines of well-formed 4-line FASTQ."""
    lines = text.split("\n")
    return [lines[i] for i in range(1, len(lines) - 1, 4)]
