"""Seeded synthetic inputs (no network: enwik8/9 are not available here or on the GPU box).

text(n, seed): enwik-class synthetic text -- a Zipf word model with per-article topic
  words, punctuation, paragraph breaks and wiki/XML-like boilerplate, generated fully
  vectorised (token ids -> byte gather) so 1e9 bytes take seconds.  bzip2 -9 compresses it to
  roughly 0.27 of its size (enwik8: 0.29, enwik9: 0.254); bench.py reports the measured ratio.
random_bytes(n, seed): PRNG bytes standing in for /dev/urandom (8.0 bits/byte).
single_byte(n, c): n copies of byte c.
"""
import numpy as np

_COMMON = ("the and of in to a is was for on as by with he that at from his it an were are which this be or "
           "first also new has had one their not after but who they its her two been other when there all "
           "during into school time may years more most only over city some world would where later up such "
           "used many can state about national out known university united then made film season team "
           "under between war american").split()

_BOILER = [b"</text>\n  </revision>\n</page>\n<page>\n  <title>", b"</title>\n  <id>",
           b"</id>\n  <revision>\n    <id>", b"</id>\n    <timestamp>2006-0", b"Z</timestamp>\n    <contributor>\n"
           b"      <username>", b"</username>\n    </contributor>\n    <text xml:space=\"preserve\">",
           b"[[Category:", b"]]\n", b"{{cite web |url=http://www.", b".org |title=", b"}} ", b"'''", b"''' ",
           b"\n\n== ", b" ==\n", b"[[", b"]] "]


_SYL = ("ing er ed es al an at en in on or re ar ic ti ent ion ter tion con com pro per ver der "
        "ly ty ry ble ful less ness ment able ist ism ous ive ate ize ist ure ance ence ical "
        "st th sh ch br cr dr fr gr pr tr bl cl fl gl pl sl sp sc sk sm sn sw tw wh qu "
        "a e i o u ai ea ee ie oa oo ou ay ey "
        "b c d f g h j k l m n p r s t v w x y z").split()


def _vocab(rng, size):
    sy = np.array(_SYL)
    ps = np.linspace(3.0, 1.0, len(sy))
    ps = ps / ps.sum()
    words = [w.encode() for w in _COMMON]
    seen = set(words)
    while len(words) < size:
        k = int(rng.choice([1, 2, 2, 3, 3, 3, 4]))
        w = "".join(rng.choice(sy, size=k, p=ps))
        if len(w) < 3:
            continue
        if rng.random() < 0.1:
            w = w.capitalize()
        b = w.encode()
        if b not in seen:
            seen.add(b)
            words.append(b)
    return words


class _TextModel:
    def __init__(self, seed):
        rng = np.random.default_rng(seed)
        words = _vocab(rng, 40000)
        V = len(words)
        toks = []
        for w in words:
            toks += [w + b" ", w + b", ", w + b". ", w + b".\n\n"]
        bstart = len(toks)
        toks += _BOILER
        lens = np.array([len(t) for t in toks], dtype=np.int64)
        self.flat = np.frombuffer(b"".join(toks), dtype=np.uint8)
        self.start = np.concatenate([[0], np.cumsum(lens)[:-1]])
        self.lens = lens
        r = np.arange(1, V + 1, dtype=np.float64)
        z = 1.0 / r ** 1.1
        self.cdf = np.cumsum(z / z.sum())
        self.V = V
        self.bstart = bstart


def text(n: int, seed: int = 0x5EED0001) -> bytes:
    m = _TextModel(seed)
    rng = np.random.default_rng(seed + 1)
    out = np.empty(n, dtype=np.uint8)
    pos = 0
    while pos < n:
        ntok = 1 << 21
        ids = np.searchsorted(m.cdf, rng.random(ntok))
        ids = np.minimum(ids, m.V - 1)
        # topic locality: articles of ~2500 tokens reuse 40 article-specific words
        art = np.arange(ntok) // 2500
        topic = np.searchsorted(m.cdf, rng.random((art[-1] + 1, 40)) * 0.35 + 0.6)
        use = rng.random(ntok) < 0.18
        ids = np.where(use, topic[art, rng.integers(0, 40, ntok)], ids)
        ids = np.minimum(ids, m.V - 1)
        # punctuation variants
        pr = rng.random(ntok)
        var = np.where(pr < 0.06, 1, np.where(pr < 0.105, 2, np.where(pr < 0.11, 3, 0)))
        tok = ids * 4 + var
        # boilerplate: article frames, categories, citations, links, headings
        k = rng.random(ntok)
        tok = np.where(k < 0.012, m.bstart + 15, tok)  # "[[" link open
        tok = np.where((k >= 0.012) & (k < 0.024), m.bstart + 16, tok)
        tok = np.where((k >= 0.024) & (k < 0.026), m.bstart + 13, tok)
        tok = np.where((k >= 0.026) & (k < 0.028), m.bstart + 14, tok)
        tok = np.where((k >= 0.028) & (k < 0.03), m.bstart + 8 + rng.integers(0, 3, ntok), tok)
        frame = (np.arange(ntok) % 2500) < 6
        tok = np.where(frame, m.bstart + (np.arange(ntok) % 2500), tok)
        lens = m.lens[tok]
        ends = np.cumsum(lens)
        total = int(ends[-1])
        take = min(total, n - pos)
        cnt = int(np.searchsorted(ends, take, side="left")) + 1
        tok, lens, ends = tok[:cnt], lens[:cnt], ends[:cnt]
        starts_out = ends - lens
        idx = np.repeat(m.start[tok] - starts_out, lens) + np.arange(int(ends[-1]))
        chunk = m.flat[idx]
        out[pos:pos + take] = chunk[:take]
        pos += take
    return out.tobytes()


def random_bytes(n: int, seed: int = 0x5EED0005) -> bytes:
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8).tobytes()


def single_byte(n: int, c: int = 0x61) -> bytes:
    return bytes([c]) * n
