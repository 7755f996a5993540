"""Multi-GPU scaling: data parallel over independent instances (dp.py) and D-sharding (dshard.py)."""
