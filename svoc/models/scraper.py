"""Comment scraper for the sentiment oracles' corpus (client/scraper.py:1-101, hn_scraper.js).

The reference drives headless Firefox through Selenium to https://news.ycombinator.com/newcomments,
runs a 9-line script that returns the trimmed ``textContent`` of every ``div.commtext.c00``, appends
them to ``data/db.sqlite`` (table ``comments``) and sleeps ``--rate`` seconds (default 10 min), first
waiting out what is left of the interval since the newest stored comment.

Here the page is fetched with ``urllib`` (no browser: the comment text is in the served HTML) and
parsed with the standard library's HTML parser.  ``source`` may also be a local ``.html`` file --
there is no network on the GPU boxes, so the tests and offline runs feed saved pages.  The SQLite
schema and the window reader are ``svoc/models/corpus.py``'s (shared with the CLI).

    python -m svoc.models.scraper --db data/db.sqlite --rate 600           # live, every 10 minutes
    python -m svoc.models.scraper --db db.sqlite --source page.html --once  # one offline pass
"""
from __future__ import annotations

import argparse
import datetime as _dt
import os
import sqlite3
import threading
import time
import urllib.request
from html.parser import HTMLParser
from typing import Callable, List, Optional

from . import corpus

URL = "https://news.ycombinator.com/newcomments"     # client/scraper.py:19
DEFAULT_REFRESH_INTERVAL = 10 * 60                     # client/scraper.py:21
_VOID = {"area", "base", "br", "col", "embed", "hr", "img", "input", "link", "meta", "source", "track", "wbr"}


class CommentExtractor(HTMLParser):
    """Text of every element whose class list holds both ``commtext`` and ``c00`` (the selector
    ``div.commtext.c00`` of hn_scraper.js: top-level-colour comments), like ``textContent``: all
    descendant text concatenated, entities decoded, then stripped."""

    def __init__(self, classes=("commtext", "c00"), tag: Optional[str] = "div"):
        super().__init__(convert_charrefs=True)
        self.want, self.tag = set(classes), tag
        self.comments: List[str] = []
        self._depth = 0            # > 0 while inside a matching element (nesting depth)
        self._buf: List[str] = []

    def handle_starttag(self, tag, attrs):
        if tag in _VOID:
            return
        if self._depth:
            self._depth += 1
            return
        cls = set((dict(attrs).get("class") or "").split())
        if self.want <= cls and (self.tag is None or tag == self.tag):
            self._depth, self._buf = 1, []

    def handle_endtag(self, tag):
        if tag in _VOID or not self._depth:
            return
        self._depth -= 1
        if self._depth == 0:
            self.comments.append("".join(self._buf).strip())

    def handle_data(self, data):
        if self._depth:
            self._buf.append(data)


def extract_comments(html: str) -> List[str]:
    p = CommentExtractor()
    p.feed(html)
    p.close()
    return p.comments


def fetch_html(source: str, timeout: float = 10.0) -> str:
    """A URL (http/https) or a local file path."""
    if source.startswith(("http://", "https://")):
        req = urllib.request.Request(source, headers={"User-Agent": "svoc-scraper/1.0"})
        with urllib.request.urlopen(req, timeout=timeout) as r:   # noqa: S310 (fixed scheme check above)
            return r.read().decode(r.headers.get_content_charset() or "utf-8", errors="replace")
    with open(source, encoding="utf-8", errors="replace") as f:
        return f.read()


def scrape_once(conn: sqlite3.Connection, source: str = URL, timeout: float = 10.0) -> List[str]:
    """scrap + save_to_db (client/scraper.py:35-42,57-62): a failed fetch stores nothing."""
    try:
        comments = extract_comments(fetch_html(source, timeout))
    except OSError:
        comments = []
    if comments:
        corpus.save_to_db(conn, comments)
    return comments


def seconds_to_wait(conn: sqlite3.Connection, refresh_interval: float, now: Optional[_dt.datetime] = None) -> float:
    """What is left of the refresh interval since the newest stored comment (client/scraper.py:78-85);
    timestamps are UTC ``%Y-%m-%d %H:%M:%S`` as corpus.save_to_db writes them."""
    last = corpus.get_last_comment_time(conn)
    if last is None:
        return 0.0
    now = now or _dt.datetime.now(_dt.timezone.utc).replace(tzinfo=None)
    elapsed = (now - _dt.datetime.strptime(last, "%Y-%m-%d %H:%M:%S")).total_seconds()
    return max(0.0, refresh_interval - elapsed)


def run(db_path: str, refresh_interval: float = DEFAULT_REFRESH_INTERVAL, source: str = URL,
        stop: Optional[threading.Event] = None, max_passes: Optional[int] = None,
        log: Callable[[str], None] = print) -> int:
    """The scraper service (client/scraper.py:74-94): wait out the interval, then scrape every
    ``refresh_interval`` seconds until ``stop`` is set or ``max_passes`` passes ran.  Returns the
    number of comments stored."""
    stop = stop or threading.Event()
    conn = corpus.init_db(db_path)
    stored, passes = 0, 0
    try:
        wait = seconds_to_wait(conn, refresh_interval)
        if wait > 0:
            log(f"<scraper> Please wait: {wait:.0f} seconds")
            if stop.wait(wait):
                return stored
        while not stop.is_set():
            got = scrape_once(conn, source)
            stored += len(got)
            passes += 1
            log(f"<scraper> - {_dt.datetime.now()} fetched {len(got)} comments")
            if max_passes is not None and passes >= max_passes:
                break
            stop.wait(refresh_interval)
    finally:
        conn.close()
    return stored


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="comment scraper (client/scraper.py)")
    ap.add_argument("--rate", type=float, default=DEFAULT_REFRESH_INTERVAL, help="refresh interval in seconds")
    ap.add_argument("--db", default=os.path.join("data", "db.sqlite"))
    ap.add_argument("--source", default=URL, help="URL or saved .html page")
    ap.add_argument("--once", action="store_true", help="one pass, no initial wait")
    a = ap.parse_args(argv)
    os.makedirs(os.path.dirname(os.path.abspath(a.db)), exist_ok=True)
    if a.once:
        conn = corpus.init_db(a.db)
        got = scrape_once(conn, a.source)
        conn.close()
        print(f"<scraper> stored {len(got)} comments")
        return 0
    print(f"<scraper> started with a refresh rate of {a.rate} seconds")
    try:
        run(a.db, a.rate, a.source)
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
