"""Test helper: mirror parameter objects (uptune_amd.manipulator) -> oracle
Param lists, and back."""
from oracle.space import BOOL, ENUM, FLOAT, INT, LOGINT, PERM, POW2, Param


def oracle_space(manip):
    out = []
    for p in manip.params:
        cls = type(p).__name__
        if cls == "FloatParameter":
            out.append(Param(p.name, FLOAT, p.min_value, p.max_value))
        elif cls == "IntegerParameter":
            out.append(Param(p.name, INT, p.min_value, p.max_value))
        elif cls == "LogIntegerParameter":
            out.append(Param(p.name, LOGINT, int(p.min_value), int(p.max_value)))
        elif cls == "PowerOfTwoParameter":
            out.append(Param(p.name, POW2, p.min_value, p.max_value))
        elif cls == "BooleanParameter":
            out.append(Param(p.name, BOOL))
        elif cls == "EnumParameter":
            out.append(Param(p.name, ENUM, options=list(p.options)))
        elif cls == "PermutationParameter":
            out.append(Param(p.name, PERM, options=list(p._items)))
        else:
            raise TypeError(cls)
    return out


def to_manip(space):
    from uptune_amd.manipulator import (BooleanParameter, ConfigurationManipulator, EnumParameter, FloatParameter,
                                        IntegerParameter, LogIntegerParameter, PermutationParameter,
                                        PowerOfTwoParameter)
    m = ConfigurationManipulator()
    for p in space:
        if p.kind == FLOAT:
            m.add_parameter(FloatParameter(p.name, p.lo, p.hi))
        elif p.kind == INT:
            m.add_parameter(IntegerParameter(p.name, p.lo, p.hi))
        elif p.kind == LOGINT:
            m.add_parameter(LogIntegerParameter(p.name, p.lo, p.hi))
        elif p.kind == POW2:
            m.add_parameter(PowerOfTwoParameter(p.name, p.lo, p.hi))
        elif p.kind == BOOL:
            m.add_parameter(BooleanParameter(p.name))
        elif p.kind == ENUM:
            m.add_parameter(EnumParameter(p.name, p.options))
        elif p.kind == PERM:
            m.add_parameter(PermutationParameter(p.name, p.options))
    return m
