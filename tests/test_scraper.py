"""Comment scraper (svoc/models/scraper.py vs client/scraper.py + hn_scraper.js) on a saved page.

The fixture is hand-written markup in the shape of the newcomments page (no network here): the
selector ``div.commtext.c00`` keeps top-level-colour comments only, textContent keeps nested text
and decodes entities, and the strings are trimmed."""
import datetime as dt
import threading

from svoc.models import corpus, scraper

PAGE = """<html><body><table>
<tr class="athing comtr"><td><div class="comment">
  <div class="commtext c00">  First comment with a <a href="x">link</a> &amp; an entity.<p>Second paragraph.</p>  </div>
</div></td></tr>
<tr class="athing comtr"><td><div class="comment">
  <div class="commtext c5a">Faded (downvoted) comment: not c00.</div>
</div></td></tr>
<tr><td><span class="commtext c00">A span, not a div.</span></td></tr>
<tr class="athing comtr"><td><div class="comment">
  <div class="c00 commtext extra">Class order does not matter<br>and void tags <img src="a.png"> are skipped.<div>nested div</div></div>
</div></td></tr>
</table></body></html>"""


def test_extract_matches_selector_and_text_content():
    got = scraper.extract_comments(PAGE)
    assert got == [
        "First comment with a link & an entity.Second paragraph.",
        "Class order does not matterand void tags  are skipped.nested div",
    ]


def test_scrape_once_from_saved_page(tmp_path):
    page = tmp_path / "newcomments.html"
    page.write_text(PAGE, encoding="utf-8")
    conn = corpus.init_db(str(tmp_path / "db.sqlite"))
    got = scraper.scrape_once(conn, str(page))
    assert len(got) == 2
    rows = conn.execute("SELECT comment FROM comments ORDER BY id").fetchall()
    assert [r[0] for r in rows] == got
    # a source that cannot be read stores nothing (the reference's scrap returns [] on failure)
    assert scraper.scrape_once(conn, str(tmp_path / "missing.html")) == []
    assert conn.execute("SELECT COUNT(id) FROM comments").fetchone()[0] == 2


def test_wait_rule(tmp_path):
    conn = corpus.init_db(str(tmp_path / "db.sqlite"))
    assert scraper.seconds_to_wait(conn, 600) == 0.0           # empty corpus: scrape at once
    corpus.save_to_db(conn, ["x"], timestamp="2026-01-01 00:00:00")
    now = dt.datetime(2026, 1, 1, 0, 4, 0)
    assert scraper.seconds_to_wait(conn, 600, now) == 360.0     # 4 of 10 minutes elapsed
    assert scraper.seconds_to_wait(conn, 600, dt.datetime(2026, 1, 1, 1)) == 0.0


def test_run_loop_passes_and_stop(tmp_path):
    page = tmp_path / "p.html"
    page.write_text(PAGE, encoding="utf-8")
    db = str(tmp_path / "db.sqlite")
    logs = []
    n = scraper.run(db, refresh_interval=0.0, source=str(page), max_passes=3, log=logs.append)
    assert n == 6 and len(logs) == 3
    conn = corpus.init_db(db)
    assert conn.execute("SELECT COUNT(id) FROM comments").fetchone()[0] == 6
    # the interval since the newest comment has not elapsed: the loop waits and can be stopped
    stop = threading.Event()
    t = threading.Thread(target=scraper.run, args=(db, 3600.0, str(page), stop), kwargs=dict(log=logs.append))
    t.start()
    stop.set()
    t.join(timeout=10)
    assert not t.is_alive()
    assert conn.execute("SELECT COUNT(id) FROM comments").fetchone()[0] == 6


def test_cli_scraper_uses_source(tmp_path):
    from svoc.cli import Client
    page = tmp_path / "p.html"
    page.write_text(PAGE, encoding="utf-8")
    cl = Client(db_path=str(tmp_path / "db.sqlite"), scraper_source=str(page))
    n0 = cl.conn.execute("SELECT COUNT(id) FROM comments").fetchone()[0]
    cl.query("scraper on")
    cl.query("fetch")
    rows = cl.conn.execute("SELECT comment FROM comments WHERE id > ?", (n0,)).fetchall()
    assert [r[0] for r in rows] == scraper.extract_comments(PAGE)
    cl.close()
