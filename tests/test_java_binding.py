"""The Java FFM binding (java/src/main/java/io/scalecube/cluster/sim/SwimHip.java) against the C ABI, without a JDK.

This image has no JDK, so the Java sources cannot be compiled here. What can go stale silently is the
struct layout and the symbol names; both are checked against the ctypes mirror of include/swimhip.h, which the rest of
the suite exercises on the real library."""
import ctypes as C
import re
from pathlib import Path

from swimhip import _abi

JAVA = Path(__file__).resolve().parent.parent / "java" / "src" / "main" / "java" / "io" / "scalecube" / "cluster" / "sim"


def java_layout(name):
    text = (JAVA / "SwimHip.java").read_text()
    body = re.search(rf"static final MemoryLayout {name} =\s*MemoryLayout\.structLayout\((.*?)\);\n", text, re.S).group(1)
    fields = []
    for m in re.finditer(r"(JAVA_INT|JAVA_LONG)\.withName\(\"(\w+)\"\)|sequenceLayout\((\d+), JAVA_INT\)\.withName"
                         r"\(\"(\w+)\"\)|paddingLayout\((\d+)\)", body):
        if m.group(1):
            fields.append((m.group(2), 4 if m.group(1) == "JAVA_INT" else 8))
        elif m.group(3):
            fields.append((m.group(4), 4 * int(m.group(3))))
        else:
            fields.append(("<pad>", int(m.group(5))))
    return fields


def check(name, struct):
    off = 0
    layout = java_layout(name)
    for fname, size in layout:
        if fname != "<pad>":
            assert getattr(struct, fname).offset == off, (name, fname, off)
            assert getattr(struct, fname).size == size, (name, fname, size)
        off += size
    assert off == C.sizeof(struct), (name, off, C.sizeof(struct))
    assert [f for f, _ in layout if f != "<pad>"] == [f for f, _ in struct._fields_]


def test_config_layout():
    check("CONFIG", _abi.SwimConfig)


def test_member_config_layout():
    check("MEMBER_CONFIG", _abi.SwimMemberConfig)


def test_event_layout():
    check("EVENT", _abi.SwimEvent)


def test_bound_symbols_exist_in_the_abi():
    text = (JAVA / "SwimHip.java").read_text()
    names = set(re.findall(r'fn\("(swim_\w+)"', text))
    assert names and names <= set(_abi.SIGNATURES), names - set(_abi.SIGNATURES)
