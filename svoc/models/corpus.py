"""Comment corpus: synthetic HN-like comments, a deterministic tokenizer and the reference's SQLite
window reader.

The reference scrapes Hacker News with Selenium into ``data/db.sqlite`` (client/scraper.py:44-94;
schema ``comments(id INTEGER PRIMARY KEY, comment TEXT, timestamp TEXT)``) and the oracle reads a
window of 30 comments starting at a position that advances by PREDICTION_WINDOW = 50 and wraps
(client/oracle_scheduler.py:44-69).  There is no network here, so comments are generated from a
seeded word model; the SQLite layer keeps the reference schema and window semantics so a real
scraped database can be dropped in.
"""
from __future__ import annotations

import datetime as _dt
import hashlib
import random
import sqlite3
from typing import List, Sequence, Tuple

import torch

PREDICTION_WINDOW = 50       # client/common.py:15
WINDOW_SIZE = 30             # LIMIT 30 (oracle_scheduler.py:62)
BOOTSTRAPING_SUBSET = 10     # client/common.py:16

_WORDS = ("the a this that it is was not very really quite so just still rust python gpu cpu compiler "
          "startup funding market model paper code bug fix release open source company hiring remote "
          "love hate great terrible amazing awful sorry worried excited hopeful angry annoyed nervous "
          "optimistic regret apologize thrilled anxious furious irritated glad happy sad fear think "
          "believe argue agree disagree because but and or if when then however although").split()


_MOODS = {
    "optimism": "hopeful promising bright future improve better optimistic confident upside growth".split(),
    "anger": "furious outraged angry rage unacceptable disgrace hostile livid scandal".split(),
    "annoyance": "annoying irritating tedious again useless bloated slow broken meh".split(),
    "excitement": "excited amazing wow incredible launch thrilled awesome finally breakthrough".split(),
    "nervousness": "worried nervous anxious risky afraid uncertain scary concerned fragile".split(),
    "remorse": "sorry regret apologize mistake my fault should have ashamed unfortunately".split(),
}


def synthetic_comments(n: int, seed: int = 0) -> List[str]:
    """HN-like comments with a latent mood: each comment mixes neutral tech words with the words of
    one dominant emotion (so even a random-init encoder sees systematically different inputs)."""
    rng = random.Random(seed)
    moods = list(_MOODS)
    out = []
    for _ in range(n):
        k = rng.randint(8, 60)
        mood = _MOODS[rng.choice(moods)]
        share = rng.uniform(0.1, 0.7)
        words = [rng.choice(mood) if rng.random() < share else rng.choice(_WORDS) for _ in range(k)]
        out.append(" ".join(words).capitalize() + ".")
    return out


def tokenize(texts: Sequence[str], seq_len: int = 128, vocab: int = 50265, bos: int = 0, eos: int = 2,
             pad: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """Deterministic hashed word-level tokenizer -> (ids [B, S], attention_mask [B, S])."""
    ids = torch.full((len(texts), seq_len), pad, dtype=torch.int64)
    mask = torch.zeros((len(texts), seq_len), dtype=torch.int64)
    for i, t in enumerate(texts):
        toks = [bos]
        for w in t.lower().split():
            h = int.from_bytes(hashlib.blake2s(w.encode(), digest_size=4).digest(), "little")
            toks.append(3 + h % (vocab - 3))
        toks = toks[: seq_len - 1] + [eos]
        ids[i, : len(toks)] = torch.tensor(toks)
        mask[i, : len(toks)] = 1
    return ids, mask


def synthetic_token_batch(B: int, S: int, vocab: int, gen: torch.Generator, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Device-side synthetic token ids with random lengths (for the throughput bench)."""
    ids = torch.randint(3, vocab, (B, S), generator=gen, device=device)
    lens = torch.randint(S // 4, S + 1, (B,), generator=gen, device=device)
    mask = (torch.arange(S, device=device)[None] < lens[:, None]).to(torch.int64)
    ids = torch.where(mask.bool(), ids, torch.ones_like(ids))
    ids[:, 0] = 0
    return ids, mask


# ---- SQLite (client/scraper.py:44-72, oracle_scheduler.py:44-69) ------------------------------

def init_db(path: str) -> sqlite3.Connection:
    conn = sqlite3.connect(path, check_same_thread=False)   # callers serialise access (cli.Client lock)
    conn.execute("CREATE TABLE IF NOT EXISTS comments (id INTEGER PRIMARY KEY AUTOINCREMENT, "
                 "comment TEXT NOT NULL, timestamp TEXT NOT NULL)")
    conn.commit()
    return conn


def save_to_db(conn: sqlite3.Connection, comments: Sequence[str], timestamp: str | None = None) -> None:
    ts = timestamp or _dt.datetime.utcnow().strftime("%Y-%m-%d %H:%M:%S")
    conn.executemany("INSERT INTO comments (comment, timestamp) VALUES (?, ?)", [(c, ts) for c in comments])
    conn.commit()


def get_last_comment_time(conn: sqlite3.Connection):
    row = conn.execute("SELECT timestamp FROM comments ORDER BY id DESC LIMIT 1").fetchone()
    return row[0] if row else None


def read_window_from_db(conn: sqlite3.Connection, position: int) -> Tuple[List[str], List[str], int]:
    """oracle_scheduler.py:44-69: advance by 50, wrap, read 30 comments from id >= position."""
    n = conn.execute("SELECT COUNT(id) FROM comments LIMIT 1").fetchone()[0]
    if n == 0:
        return [], [], 0
    position = (position + PREDICTION_WINDOW) % n
    if position + PREDICTION_WINDOW >= n:
        position = 0
    rows = conn.execute("SELECT comment, timestamp FROM comments WHERE id >= ? ORDER BY id ASC LIMIT ?",
                        (position, WINDOW_SIZE)).fetchall()
    return [r[0] for r in rows], [r[1] for r in rows], position
