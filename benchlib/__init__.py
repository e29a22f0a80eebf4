"""bench.py's modules (the harness that measures the engine; not part of the product)."""
