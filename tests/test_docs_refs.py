"""Every measurement file the documentation cites exists in the tree: `profiles/...` paths in
DESIGN.md, README.md and INTEGRATION.md (globs such as `profiles/r03_v26_*` must match something,
and `r0N_...` file names quoted without the directory are looked up under profiles/)."""

import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ("DESIGN.md", "README.md", "INTEGRATION.md")


def cited(doc):
    txt = open(os.path.join(ROOT, doc)).read()
    out = set()
    for m in re.finditer(r"`(profiles/[^`\s]+)`", txt):
        out.add(m.group(1).rstrip(".,;:)"))
    for m in re.finditer(r"`(r0[0-9]_[^`\s]+\.(?:json|log|csv))`", txt):
        out.add("profiles/" + m.group(1))
    # range notation (r03_v21..v23_...) names a series, not one file
    return sorted(p for p in out if ".." not in p)


@pytest.mark.parametrize("doc", DOCS)
def test_cited_profiles_exist(doc):
    missing = []
    for p in cited(doc):
        pat = re.sub(r"\{[^}]*\}", "*", p)
        if not glob.glob(os.path.join(ROOT, pat)):
            missing.append(p)
    assert not missing, f"{doc} cites missing files: {missing}"


def test_boundary_header_states_the_model_limits():
    """include/zbot.h tells a binding maintainer the collider limits: the number it
    states is ZB_MAX_GEOM of include/zbot_model.h, and the model version it names is ZB_MODEL_VERSION."""
    hdr = open(os.path.join(ROOT, "include", "zbot.h")).read()
    mdl = open(os.path.join(ROOT, "include", "zbot_model.h")).read()
    max_geom = int(re.search(r"#define ZB_MAX_GEOM\s+(\d+)", mdl).group(1))
    version = int(re.search(r"#define ZB_MODEL_VERSION\s+(\d+)", mdl).group(1))
    m = re.search(r"1 to (\d+) floor colliders\s*\*?\s*\(ZB_MAX_GEOM, model version (\d+)", hdr)
    assert m, "zbot.h no longer states the floor-collider limit"
    assert int(m.group(1)) == max_geom and int(m.group(2)) == version
    assert "convex meshes" in hdr and "npair" in hdr
