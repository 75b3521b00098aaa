"""ORACLE -- test infrastructure only (CPU restatement of the reference's Groth16 path).

Importable only from ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg, and there only as the checker. The product package ``zebra_amd``
never imports it; see DESIGN.md "Oracle".
"""
