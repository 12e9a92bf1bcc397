"""History ingestion (uptune_amd/history.py) and the ut.params.json schema
compiler (uptune_amd/schema.py) -- SURVEY.md §8(f) rows 1 and 2.  CPU tests;
the device-side halves are in tests/test_gpu_history.py."""
import json
import os
import sqlite3

import pytest

from uptune_amd import _lib as L
from uptune_amd import history as H
from uptune_amd import schema as S


def test_opentuner_db_result_hashes(golden_dir):
    db = os.path.join(golden_dir, "tutorial_opentuner.db")
    rows = json.load(open(os.path.join(golden_dir, "tutorial_db_hashes.json")))["rows"]
    got = H.opentuner_result_hashes(db)
    # 9 configurations, 7 of them with a Result (has_results, driver.py:157-158)
    assert len(got) == 7 and len(set(got)) == 7
    assert set(got) <= {r["hash"] for r in rows}
    assert H.opentuner_result_hashes(db, tuning_run_id=1) == got
    assert H.opentuner_result_hashes(db, tuning_run_id=2) == []
    assert H.opentuner_result_hashes("sqlite:///" + db) == got


def test_global_db_hashes(tmp_path):
    path = str(tmp_path / "global")
    con = sqlite3.connect(path)
    # GlobalResult's table (database/globalmodels.py:22-36)
    con.execute("CREATE TABLE global_result (id INTEGER PRIMARY KEY, epoch INTEGER, node INTEGER, "
                "hashv VARCHAR(64), data BLOB, time DATETIME, technique VARCHAR, result FLOAT, was_the_best BOOLEAN)")
    hs = ["%064x" % (i * 7919) for i in range(5)]
    for i, h in enumerate(hs):
        con.execute("INSERT INTO global_result (epoch, node, hashv, result) VALUES (?, ?, ?, ?)", (0, i % 2, h, 1.0))
    con.commit()
    con.close()
    assert H.global_result_hashes(path) == hs


def test_read_archive(golden_dir):
    # samples/causal-graph/poly.py: x, a in (2, 15); y, b in (2, 12)
    m = S.create_params([["IntegerParameter", "x", [2, 15]], ["IntegerParameter", "y", [2, 12]],
                         ["IntegerParameter", "a", [2, 15]], ["IntegerParameter", "b", [2, 12]]])
    from uptune_amd.manipulator import compile_space
    cfgs = H.read_archive(os.path.join(golden_dir, "causal_archive.csv"), compile_space(m))
    assert len(cfgs) == 50
    assert cfgs[0] == {"x": 14, "y": 4, "a": 2, "b": 9}
    assert all(2 <= c["x"] <= 15 and 2 <= c["y"] <= 12 for c in cfgs)


def test_read_archive_enum_codes_and_perms(tmp_path):
    tokens = [["EnumParameter", "opt", ["-O2", "-O3", "-Os"]], ["PermutationParameter", "order", [0, 1, 2]],
              ["BooleanParameter", "flag", ""], ["FloatParameter", "f", [0, 1]]]
    spec = S.compile_space(S.create_params(tokens))
    p = tmp_path / "ut.archive.csv"
    p.write_text("opt,order,flag,f,qor\n2,\"[2, 0, 1]\",True,0.25,3\n-Os,\"[0, 1, 2]\",0,0.5,1\n")
    cfgs = H.read_archive(str(p), spec, S.enum_codes(tokens))
    assert cfgs == [{"opt": "-O3", "order": [2, 0, 1], "flag": True, "f": 0.25},
                    {"opt": "-Os", "order": [0, 1, 2], "flag": False, "f": 0.5}]


def test_params_json_stages(tmp_path):
    stage0 = [["IntegerParameter", "x", [2, 15]], ["EnumParameter", "mode", ["a", "b"]],
              ["FloatParameter", "lr", [0.001, 0.1]], ["LogIntegerParameter", "tile", [1, 4096]],
              ["PowerOfTwoParameter", "vec", [1, 64]], ["BooleanParameter", "unroll", ""],
              ["PermutationParameter", "order", ["i", "j", "k"]]]
    stage1 = [["IntegerParameter", "y", [0, 3]]]
    path = tmp_path / "ut.params.json"
    path.write_text(json.dumps([stage0, stage1]))     # report.update appends one list per stage
    ms = S.load_params_json(str(path))
    assert [len(m.params) for m in ms] == [7, 1]
    spec = S.compile_stage(str(path), 0)
    assert [p.kind for p in spec.params] == [L.UT_INT, L.UT_ENUM, L.UT_FLOAT, L.UT_LOGINT, L.UT_POW2, L.UT_BOOL,
                                             L.UT_PERM]
    assert spec.ncols == 6 + 3 and spec.n_features == 1 + 2 + 1 + 1 + 1 + 1 + 3
    assert [p.col for p in spec.params] == [0, 1, 2, 3, 4, 5, 6]
    # a bare token list is one stage
    path.write_text(json.dumps(stage0))
    assert len(S.load_params_json(str(path))) == 1
    assert S.enum_codes(stage0) == {"mode": {1: "a", 2: "b"}}
    with pytest.raises(ValueError):
        S.create_params([["TuneFoo", "z", [0, 1]]])
