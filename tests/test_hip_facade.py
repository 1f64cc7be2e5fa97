"""ops/hip.py is a facade over ops/_hip/*: every top-level name of a part is reachable as ``hip.X``, and
``hip.X = v`` rebinds X in the part that owns it (the parts read their flags as module globals)."""
import ast
import os

import pytest

PARTS = ("common", "shadows", "gemm", "streams", "pool", "convbn", "misc", "adam")
ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "pytorch_imageclassification_distributed_amd", "ops", "_hip")


def _top_level(path):
    names = set()
    for nd in ast.parse(open(path).read()).body:
        if isinstance(nd, (ast.FunctionDef, ast.ClassDef)):
            names.add(nd.name)
        elif isinstance(nd, ast.Assign):
            for t in nd.targets:
                if isinstance(t, ast.Name):
                    names.add(t.id)
                elif isinstance(t, ast.Tuple):
                    names |= {e.id for e in t.elts if isinstance(e, ast.Name)}
        elif isinstance(nd, ast.AnnAssign) and isinstance(nd.target, ast.Name):
            names.add(nd.target.id)
    return names - {"_OWNED"}


def _owned(path):
    for nd in ast.parse(open(path).read()).body:
        if isinstance(nd, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "_OWNED" for t in nd.targets):
            return set(ast.literal_eval(nd.value))
    return set()


@pytest.mark.parametrize("part", PARTS)
def test_every_top_level_name_is_owned(part):
    path = os.path.join(ROOT, part + ".py")
    assert _top_level(path) == _owned(path)


def test_names_are_unique_across_parts():
    seen = {}
    for part in PARTS:
        for n in _owned(os.path.join(ROOT, part + ".py")):
            assert n not in seen, (n, seen.get(n), part)
            seen[n] = part


def test_flag_writes_reach_the_owner():
    try:
        from pytorch_imageclassification_distributed_amd.ops import hip
        from pytorch_imageclassification_distributed_amd.ops._hip import gemm, convbn
    except Exception as e:  # the extension is not built here
        pytest.skip(f"HIP extension not importable: {e}")
    keep = hip.DEEP_FORCE, hip.RELU_MASK
    try:
        hip.DEEP_FORCE = 3
        hip.RELU_MASK = not keep[1]
        assert gemm.DEEP_FORCE == 3 and hip.DEEP_FORCE == 3
        assert convbn.RELU_MASK == (not keep[1]) and hip.RELU_MASK == (not keep[1])
    finally:
        hip.DEEP_FORCE, hip.RELU_MASK = keep
    assert gemm.DEEP_FORCE == keep[0]
    assert hip.conv_bn_act is convbn.conv_bn_act
