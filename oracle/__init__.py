"""Parity oracle — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference path (snarkjs/ffjavascript Groth16 over BN254, circomlib
Poseidon).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import, link or execute anything under ``oracle/`` — always as the
checker, never as the thing measured or shipped.  The product package never imports it.
"""
