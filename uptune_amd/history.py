"""History ingestion into the device dedup set.

The reference decides "seen before" per candidate with SQL and pandas
(SURVEY.md §8(a) a6):

  (i)   a Result row of this tuning run for the Configuration with that hash
        (SearchDriver.has_results -> results_query, driver.py:157-158,
        driverbase.py:24-43; Configuration.hash, resultsdb/models.py:120-135)
  (ii)  a GlobalResult with that hash, across instances and stages
        (GlobalResult.get, database/globalmodels.py:38-45; api.py:261)
  (iii) all-column equality with a row of ut.archive.csv (api.py:264-275)
  (iv)  an in-flight (pending) configuration

Here all four are bulk-exported once (startup / resume) and after each round
into the GPU history set, so dedup is one device probe per candidate.  The
databases are read with sqlite3 in read-only mode and only their hash
columns are touched: the pickled `data` columns are never loaded.  Archive
rows are hashed on the device (ut_hash), which makes (iii) digest equality --
the same as column equality for configs of one space.
"""
from __future__ import annotations

import ast
import csv
import sqlite3
from typing import Any, Dict, Iterable, List, Optional, Sequence

from . import _lib as L
from .manipulator import SpaceSpec


def _ro(path: str) -> sqlite3.Connection:
    if path.startswith("sqlite:///"):
        path = path[len("sqlite:///"):]
    return sqlite3.connect(f"file:{path}?mode=ro", uri=True)


def opentuner_result_hashes(db_path: str, tuning_run_id: Optional[int] = None,
                            program_id: Optional[int] = None) -> List[str]:
    """(i): hashes of configurations that have a Result (optionally of one
    tuning run / program, as results_query filters by tuning_run)"""
    q = ("SELECT DISTINCT c.hash FROM result r JOIN configuration c ON r.configuration_id = c.id "
         "WHERE c.hash IS NOT NULL")
    args: List[Any] = []
    if tuning_run_id is not None:
        q += " AND r.tuning_run_id = ?"
        args.append(int(tuning_run_id))
    if program_id is not None:
        q += " AND c.program_id = ?"
        args.append(int(program_id))
    with _ro(db_path) as con:
        return [h for (h,) in con.execute(q + " ORDER BY r.id", args)]


def global_result_hashes(db_path: str) -> List[str]:
    """(ii): GlobalResult.hashv of every row (table global_result)"""
    with _ro(db_path) as con:
        return [h for (h,) in con.execute("SELECT hashv FROM global_result WHERE hashv IS NOT NULL ORDER BY id")]


def _parse(ps, text: str, codes: Optional[Dict[int, Any]]):
    k = ps.kind
    if k == L.UT_FLOAT:
        return float(text)
    if k in (L.UT_INT, L.UT_LOGINT, L.UT_POW2):
        return int(float(text))
    if k == L.UT_BOOL:
        t = text.strip()
        if t in ("True", "False"):
            return t == "True"
        return bool(int(float(t)))
    if k == L.UT_ENUM:
        by_str = {str(o): o for o in ps.options}
        if text in by_str:
            return by_str[text]
        if codes:
            return codes[int(float(text))]
        raise ValueError(f"archive value {text!r} is not an option of enum {ps.name!r}")
    if k == L.UT_PERM:
        return list(ast.literal_eval(text))     # literals only: nothing is executed
    raise TypeError(k)


def read_archive(csv_path: str, spec: SpaceSpec, codes: Optional[Dict[Any, Dict[int, Any]]] = None
                 ) -> List[Dict[Any, Any]]:
    """(iii): the space's columns of every ut.archive.csv row as config dicts
    (extra columns -- time, features, qor, is_best -- are ignored).  `codes`
    maps integer-coded enum columns back to options (schema.enum_codes)."""
    codes = codes or {}
    out = []
    with open(csv_path, newline="") as f:
        for row in csv.DictReader(f):
            out.append({ps.name: _parse(ps, row[str(ps.name)], codes.get(ps.name)) for ps in spec.params})
    return out


def ingest_history(engine, opentuner_db: Optional[str] = None, tuning_run_id: Optional[int] = None,
                   global_db: Optional[str] = None, archive_csv: Optional[str] = None,
                   archive_codes=None, pending: Iterable[Dict[Any, Any]] = ()) -> int:
    """Add every seen configuration to the engine's device history set;
    returns the number of digests added."""
    hexes: List[str] = []
    if opentuner_db:
        hexes += opentuner_result_hashes(opentuner_db, tuning_run_id)
    if global_db:
        hexes += global_result_hashes(global_db)
    cfgs: List[Dict[Any, Any]] = list(pending)
    if archive_csv:
        cfgs += read_archive(archive_csv, engine.spec, archive_codes)
    if cfgs:
        hexes += engine.hash_configs(cfgs)
    if hexes:
        engine.history_add(hexes)
    return len(hexes)


def seen_mask(engine, cfgs: Sequence[Dict[Any, Any]]) -> List[bool]:
    """dedup verdicts for host configs (history + earlier rows of the batch)"""
    import torch
    if not len(cfgs):
        return []
    vals = torch.from_numpy(engine.spec.encode_configs(cfgs)).to(engine.device)
    return [bool(x) for x in engine.dedup(engine.hash(vals)).cpu().numpy()]
