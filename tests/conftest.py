import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ksim-gym-zbot_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def cmodel():
    from zbot_amd import compile_model

    return compile_model()


def mjcf_variant_desc():
    """The default robot written as MJCF and edited into everything the converter maps that the
    default descriptor leaves at identity: rotated inertial frames, geom-derived inertia (capsule
    arm links), a non-unit gear and an asymmetric ctrlrange."""
    import math
    import xml.etree.ElementTree as ET

    from zbot_amd.mjcf import load_mjcf, to_mjcf
    from zbot_amd.model import load_description

    root = ET.fromstring(to_mjcf(load_description()))
    root.find("default").append(ET.fromstring('<default class="arm"><geom type="capsule" density="1200" contype="0" conaffinity="0"/></default>'))
    axes = [(1, 2, 3, 25.0), (0, 1, 1, -40.0), (3, -1, 2, 70.0), (1, 0, 0, 90.0)]
    k = 0
    for b in root.iter("body"):
        name = b.get("name")
        inert = b.find("inertial")
        if name.endswith(("elbow_roll_link", "gripper_roll_link")):
            b.remove(inert)  # inertia from a capsule along the link
            b.append(ET.fromstring('<geom class="arm" size="0.012" fromto="0 0 0 0.004 0.002 -0.05"/>'))
        elif "knee" in name or "hip_pitch" in name or "shoulder_roll" in name:
            x, y, z, deg = axes[k % len(axes)]
            n = math.sqrt(x * x + y * y + z * z)
            s = math.sin(math.radians(deg) / 2)
            inert.set("quat", f"{math.cos(math.radians(deg) / 2)!r} {x / n * s!r} {y / n * s!r} {z / n * s!r}")
            k += 1
    for a in root.find("actuator"):
        if a.get("joint") == "left_knee_pitch":
            a.set("gear", "1.25")
        if a.get("joint") == "right_hip_roll":
            a.set("ctrlrange", "-0.8 1.1")
    return load_mjcf(ET.tostring(root, encoding="unicode"))


@pytest.fixture(scope="session")
def cmodel_mjcf():
    from zbot_amd import compile_model

    return compile_model(mjcf_variant_desc())


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as O

    O.build()
    return O
