"""ORACLE -- test infrastructure only (CPU restatement of the reference hot path).

Importable only from ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg. The product package never imports it. See ``refcpu.py``.
"""
