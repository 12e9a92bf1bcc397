"""The `ut.params.json` schema compiler.

uptune's profiling run records every `ut.tune(...)` call site as a token
`[ptype, name, scope]` (python/uptune/template/types.py:61-89) and appends
the token list of each stage to `ut.params.json` (report.py:57-60,
report.py:106-118: the file is a JSON list of stages).  The tuner reads it
back (api.py:104-106) and builds one ConfigurationManipulator per stage
(`create_params`, api.py:179-199).  This module does the same and hands the
manipulator to `compile_space`, which produces the device layout: SoA value
columns, inner-digest LUTs, the fixed outer hash-message template and the
name sort ranks -- so a `ut.tune()` program runs on the GPU path unchanged.

    stages = load_params_json("ut.params.json")     # [ConfigurationManipulator]
    spec   = compile_stage("ut.params.json", 0)      # SpaceSpec for ut_space_define
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Sequence

from .manipulator import (BooleanParameter, ConfigurationManipulator, EnumParameter, FloatParameter,
                          IntegerParameter, LogIntegerParameter, PermutationParameter, PowerOfTwoParameter,
                          SpaceSpec, compile_space)

PTYPES = ("IntegerParameter", "EnumParameter", "FloatParameter", "LogIntegerParameter", "PowerOfTwoParameter",
          "BooleanParameter", "PermutationParameter")


def create_params(tokens: Sequence[Sequence[Any]]) -> ConfigurationManipulator:
    """api.py:179-199: one parameter per [ptype, name, scope] token"""
    m = ConfigurationManipulator()
    for item in tokens:
        ptype, pname, prange = item
        if ptype == "IntegerParameter":
            m.add_parameter(IntegerParameter(pname, prange[0], prange[1]))
        elif ptype == "EnumParameter":
            m.add_parameter(EnumParameter(pname, prange))
        elif ptype == "FloatParameter":
            m.add_parameter(FloatParameter(pname, prange[0], prange[1]))
        elif ptype == "LogIntegerParameter":
            m.add_parameter(LogIntegerParameter(pname, prange[0], prange[1]))
        elif ptype == "PowerOfTwoParameter":
            m.add_parameter(PowerOfTwoParameter(pname, prange[0], prange[1]))
        elif ptype == "BooleanParameter":
            m.add_parameter(BooleanParameter(pname))
        elif ptype == "PermutationParameter":
            m.add_parameter(PermutationParameter(pname, prange))
        else:
            raise ValueError("unrecognized type " + str(ptype))   # api.py:198 asserts
    return m


def stages_of(doc) -> List[List[List[Any]]]:
    """a parsed ut.params.json -> token lists per stage (a bare token list is
    accepted as a single stage)"""
    if not isinstance(doc, list):
        raise ValueError("ut.params.json must hold a JSON list")
    if doc and isinstance(doc[0], list) and len(doc[0]) == 3 and isinstance(doc[0][0], str) \
            and doc[0][0] in PTYPES:
        return [doc]
    return [list(stage) for stage in doc]


def load_params_json(path: str) -> List[ConfigurationManipulator]:
    with open(path) as f:
        return [create_params(tokens) for tokens in stages_of(json.load(f))]


def compile_stage(path: str, stage: int = 0) -> SpaceSpec:
    return compile_space(load_params_json(path)[stage])


def enum_codes(tokens: Sequence[Sequence[Any]]) -> Dict[Any, Dict[int, Any]]:
    """the archive's integer codes of enum options: 1-based over the sorted
    options (ParallelTuning.training, api.py:296-300) -> {name: {code: option}}"""
    out = {}
    for ptype, pname, prange in tokens:
        if ptype == "EnumParameter":
            out[pname] = {k + 1: v for k, v in enumerate(sorted(set(prange)))}
    return out
