"""ORACLE -- TEST INFRASTRUCTURE ONLY (never imported by prodiff_amd).

numpy restatements of the reference hot path; see oracle_prodiff.py and
oracle_fastdiff.py.  Pinned against tests/golden/*.npz (reference outputs).
"""
