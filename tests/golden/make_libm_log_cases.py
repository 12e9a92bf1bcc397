"""Generate tests/golden/libm_log_non_cr.json: integers x in [2^22, 2^31)
for which this image's math.log(x) (glibc's log) is NOT the correctly rounded
natural log -- the arguments where a correctly rounded device log disagreed
with the reference in round 1.  The GPU test hashes LogInteger values at
these arguments and compares with the box's own CPython (which must agree
with the device restatement ut_core.h libm_log).  Candidates are screened with
long-double logs and confirmed with 60-digit Decimal.

    python tests/golden/make_libm_log_cases.py
"""
import json
import math
import os
from decimal import Decimal, getcontext

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main(count=256, seed=5):
    getcontext().prec = 60
    rng = np.random.default_rng(seed)
    found = []
    while len(found) < count:
        xs = rng.integers(1 << 22, 1 << 31, size=1 << 20)
        libm = np.array([math.log(float(x)) for x in xs.tolist()])
        ld = np.log(xs.astype(np.longdouble)).astype(np.float64)
        for x in xs[libm != ld].tolist():
            if math.log(x) != float(Decimal(x).ln()):
                found.append(int(x))
    found = sorted(set(found))[:count]
    with open(os.path.join(HERE, "libm_log_non_cr.json"), "w") as f:
        json.dump({"what": "x with math.log(x) != correctly rounded log(x) (glibc 2.35 __log_fma)",
                   "ints": found}, f)


if __name__ == "__main__":
    main()
