"""oracle -- CPU restatement of the reference's batch-scoring hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under uptune_amd/ imports, calls or links
this package; only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use it, and only as the checker (or as the timed CPU
baseline), never as the thing measured or shipped.

Each function cites the reference file:line it restates
(python/uptune/opentuner/search/... relative to the reference root).

Pinning (see DESIGN.md "Oracle"):
  * hash_config layout is pinned by the reference's own data: the 9
    (hash, BLOCK_SIZE) Configuration rows of
    samples/tutorials/tuneup.opentuner.db (Python-2 layout), checked in
    tests/test_oracle.py against tests/golden/tutorial_db_hashes.json;
  * SHA-256 by FIPS 180-4 vectors, Philox4x32-10 by the Random123 KATs,
    repr(float) is CPython's own repr;
  * the DE / PSO / GA operator arithmetic follows the cited lines with the
    reference's Python-`random` draws replaced by counter-based Philox draws
    (the reference itself is not reproducible under a seed, so
    parity is "identical draws -> identical outputs");
  * the GP/EI/top-k stage has NO reference implementation:
    its oracle is this package's own fp64 NumPy/SciPy code -- parity
    unpinned by the reference, pinned by the committed golden vectors.
"""
