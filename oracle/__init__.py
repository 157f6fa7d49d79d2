"""CPU restatements of the reference bloom filter (lsm/bloom.go) — TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker.  The shipped library never imports, links or executes anything under oracle/.
"""
