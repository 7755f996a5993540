"""``python -m svoc``: the reference client's CLI (client/main.py:14-74) on the local engine."""
import argparse
import sys

from .cli import DIMENSION, Client


def main(argv=None):
    ap = argparse.ArgumentParser(description="svoc oracle consensus client")
    ap.add_argument("--disable_startup_fetch", action="store_true", default=False)
    ap.add_argument("--dimension", type=int, default=DIMENSION)
    ap.add_argument("--live_mode", action="store_true", default=False)
    ap.add_argument("--scraper", action="store_true", default=False, help="scrape (or synthesise) comments on fetch")
    ap.add_argument("--scraper-source", default=None, help="URL or saved page for the scraper (svoc/models/scraper.py)")
    ap.add_argument("--rate", type=int, default=30 * 60, help="(kept for compatibility; no network)")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--mode", default="exact", choices=["exact", "fast"])
    ap.add_argument("--db", default=None, help="SQLite corpus (reference schema)")
    ap.add_argument("--encoder", default="tiny", choices=["tiny", "base"])
    ap.add_argument("--refresh", type=float, default=5.0, help="auto_fetch period in seconds (client/common.py:11)")
    ap.add_argument("-c", "--command", action="append", default=[], help="run a command and exit")
    ap.add_argument("--web", action="store_true", help="serve the browser UI instead (python -m svoc.web)")
    ap.add_argument("--port", type=int, default=8080)
    a = ap.parse_args(argv)
    if a.web:
        from .web.app import main as web_main
        args = ["--port", str(a.port), "--device", a.device, "--mode", a.mode, "--dimension", str(a.dimension),
                "--refresh", str(a.refresh)]
        args += ["--db", a.db] if a.db else []
        args += ["--scraper-source", a.scraper_source] if a.scraper_source else []
        args += ["--disable_startup_fetch"] if a.disable_startup_fetch else []
        return web_main(args)
    cl = Client(device=a.device, mode=a.mode, db_path=a.db, encoder=a.encoder, dimension=a.dimension,
                refresh_rate=a.refresh, scraper_source=a.scraper_source)
    cl.flags["scraper"] = a.scraper
    cl.flags["live_mode"] = a.live_mode
    if a.command:
        for c in a.command:
            print(cl.query(c))
        cl.close()
        return 0
    if not a.disable_startup_fetch:
        print(cl.query("resume"))
        print(cl.query("fetch"))
    while True:
        try:
            line = input("svoc> ")
        except EOFError:
            cl.close()
            return 0
        if line.strip() == "exit":
            cl.close()
            return 0
        print(cl.query(line))


if __name__ == "__main__":
    sys.exit(main())
