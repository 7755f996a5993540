"""Browser UI (FastAPI + a static page): ``python -m svoc.web``."""
