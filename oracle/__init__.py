"""Parity oracle — TEST INFRASTRUCTURE ONLY (see wavenet_ref.py header)."""
