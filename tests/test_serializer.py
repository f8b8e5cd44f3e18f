"""Scene file format: SaveScene / LoadScene (serializer.cpp:395-529).

The reference ships no scene files, so the format is pinned by its writer's
definition: nlohmann dump(4) JSON with sorted keys, object references as
indices (-1 = null), per-asset binary files with the 'TEX ' / 'MESH' /
'SPEC' headers and mz_compress (zlib) blocks behind a 4-byte size (mz_ulong
on the reference's LLP64 platform; an 8-byte size is read as well).  A
round trip must reproduce every packed buffer the integrator consumes
byte for byte, and a file written the reference's way (no vertex block, no
extension keys) must load.
"""
from __future__ import annotations

import json
import struct
import zlib

import numpy as np
import pytest

from test_ingestion import write_model


def packed(scene):
    scene.pack()
    return scene.arrays()


def assert_same_packs(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert a[k].tobytes() == b[k].tobytes(), k


@pytest.mark.parametrize("config", [1, 2, 3, 5])
def test_roundtrip_config_scenes(pt, tmp_path, config):
    s = pt.Scene.config(config)
    ref = packed(s)
    s.save(tmp_path / "scene" / "scene.json")
    t = pt.Scene.load(tmp_path / "scene" / "scene.json")
    assert t.counts() == s.counts()
    assert_same_packs(ref, packed(t))
    for x in (s, t):
        x.close()


def test_roundtrip_prefab_scene(pt, tmp_path):
    s = pt.Scene.create()
    prefab = s.load_model_as_prefab(write_model(tmp_path))
    s.instantiate_prefab(prefab)
    s.instantiate_prefab(prefab)
    ref = packed(s)
    s.save(tmp_path / "out" / "box scene.json")
    t = pt.Scene.load(tmp_path / "out" / "box scene.json")
    assert t.counts() == s.counts() and t.counts()[3] == 1
    assert_same_packs(ref, packed(t))
    for x in (s, t):
        x.close()


def test_json_layout(pt, tmp_path):
    s = pt.Scene.create()                       # CreateScene: checker plane + camera
    sph = s.create_entity(pt.ENTITY_SPHERE, position=(0, 0, 1))
    m = s.create_material(pt.MATERIAL_BASIC_METAL, "Gold", BaseColor=(1.0, 0.7, 0.3), Roughness=0.3)
    s.set_material(sph, m)
    path = tmp_path / "s" / "scene.json"
    s.save(path)
    text = path.read_text()

    pairs = []
    doc = json.loads(text, object_pairs_hook=lambda kv: (pairs.append([k for k, _ in kv]), dict(kv))[1])
    assert all(keys == sorted(keys) for keys in pairs)          # std::map order
    assert text.startswith("{\n    \"Materials\": [\n")          # dump(4)
    assert set(doc) == {"Materials", "Root", "Textures"}         # no meshes / prefabs: keys absent

    tex = doc["Textures"][0]
    assert tex == {"EnableNearestFiltering": True, "Name": "Plane Texture", "Type": 1}
    mats = doc["Materials"]
    assert mats[0]["Type"] == 0 and mats[0]["BaseTexture"] == 0
    assert set(mats[0]) == {"BaseColor", "BaseTexture", "Flags", "Name", "Opacity", "Type"}
    gold = mats[1]
    assert gold["Type"] == 1 and gold["Name"] == "Gold" and gold["SpecularTexture"] == -1
    assert gold["Roughness"] == float(np.float32(0.3))           # float -> double, shortest digits
    assert '"Roughness": 0.30000001192092896' in text
    assert '"Opacity": 1.0' in text and '"Flags": 0' in text

    root = doc["Root"]
    assert root["Type"] == 0 and root["Material"] == -1 and root["SkyboxTexture"] == -1
    kids = root["Children"]
    assert [k["Type"] for k in kids] == [4, 2, 5]               # plane, camera, sphere
    assert kids[0]["Material"] == 0 and kids[2]["Material"] == 1
    assert kids[0]["Children"] is None                           # nlohmann: untouched key -> null
    cam = kids[1]
    assert cam["Pinhole"] == {"ApertureDiameterInMM": 0.0, "FieldOfViewInDegrees": 90.0}
    assert cam["ThinLens"]["SensorSizeInMM"] == [32.0, 18.0]
    assert cam["Position"] == [0.0, 0.0, 1.0] and cam["Scale"] == [1.0, 1.0, 1.0]

    # Binary asset: MakeFileName + 'TEX ' header + size-prefixed zlib block.
    raw = (path.parent / "Plane_Texture.texture").read_bytes()
    magic, version, w, h = struct.unpack_from("<4I", raw)
    assert magic == 0x54455820 and raw[:4] == b" XET" and version == 0 and (w, h) == (2, 2)
    (n,) = struct.unpack_from("<I", raw, 16)
    assert len(raw) == 20 + n
    px = np.frombuffer(zlib.decompress(raw[20:20 + n]), np.float32).reshape(4, 4)
    assert np.array_equal(px, [[1, 1, 1, 1], [.5, .5, .5, 1], [.5, .5, .5, 1], [1, 1, 1, 1]])
    spec = (path.parent / "spectrum.dat").read_bytes()
    assert struct.unpack_from("<2I", spec) == (0x53504543, 0)
    (n,) = struct.unpack_from("<I", spec, 8)
    assert len(spec) == 12 + n
    assert len(zlib.decompress(spec[12:12 + n])) == 3 * 64 * 64 * 64 * 12
    s.close()


@pytest.mark.parametrize("value,text", [
    (1.0, "1.0"), (90.0, "90.0"), (0.5, "0.5"), (1e-3, "0.0010000000474974513"),
    (2.5e-5, "2.499999936844688e-05"), (1e-4, "9.999999747378752e-05"), (123456.0, "123456.0"),
    (-2.0, "-2.0"), (0.0, "0.0"), (3e20, "3.000000060122632e+20"),
])
def test_float_text(pt, tmp_path, value, text):
    """nlohmann prints the float's exact double in shortest round-trip digits,
    plain for decimal exponents in (-4, 15], else d.ddde+XX."""
    s = pt.Scene.empty()
    s.create_material(pt.MATERIAL_BASIC_TRANSLUCENT, "M", IOR=value)
    s.save(tmp_path / "f.json")
    doc_text = (tmp_path / "f.json").read_text()
    assert f'"IOR": {text},' in doc_text
    assert json.loads(doc_text)["Materials"][0]["IOR"] == float(np.float32(value))
    s.close()


def _compressed(data: bytes, width: int = 4) -> bytes:
    z = zlib.compress(data)
    return struct.pack("<I" if width == 4 else "<Q", len(z)) + z


@pytest.mark.parametrize("width", [4, 8])
def test_load_reference_written_files(pt, tmp_path, width):
    """Files as the reference's SaveScene writes them: no extension keys and
    a .mesh file that ends after the nodes (the reference writes no vertices);
    block sizes as a 4-byte mz_ulong (its LLP64 build) or an 8-byte one."""
    doc = {
        "Materials": [{"BaseColor": [0.8, 0.3, 0.3], "BaseTexture": -1, "Flags": 0, "Name": "Red",
                       "Opacity": 1.0, "Type": 0}],
        "Meshes": [{"Name": "Tri"}],
        "Root": {
            "Active": True, "Material": -1, "Name": "Scene", "Position": [0, 0, 0], "Rotation": [0, 0, 0],
            "Scale": [1, 1, 1], "ScatterRate": 0.0, "SkyboxBrightness": 2.0, "SkyboxTexture": -1, "Type": 0,
            "Children": [
                {"Active": True, "Children": None, "Material": 0, "Name": "Ball", "Position": [0, 0, 1],
                 "Rotation": [0, 0, 0], "Scale": [1, 1, 1], "Type": 5},
                {"Active": True, "Children": None, "Material": -1, "Name": "Cam", "Position": [0, -4, 1],
                 "Rotation": [1.5707963, 0, 0], "Scale": [1, 1, 1], "Type": 2, "CameraModel": 0,
                 "Pinhole": {"ApertureDiameterInMM": 0.0, "FieldOfViewInDegrees": 60.0},
                 "ThinLens": {"ApertureDiameterInMM": 10.0, "FocalLengthInMM": 20.0, "FocusDistance": 1.0,
                              "SensorSizeInMM": [32.0, 18.0]}},
            ],
        },
    }
    (tmp_path / "ref.json").write_text(json.dumps(doc, indent=4))
    faces = np.array([[0, 1, 2]], np.uint32)
    nodes = np.zeros(1, dtype=[("mn", "<f4", 3), ("mx", "<f4", 3), ("fb", "<u4"), ("fe", "<u4"), ("ch", "<u4")])
    nodes[0] = ((0, 0, 0), (1, 1, 0), 0, 1, 0)
    (tmp_path / "Tri.mesh").write_bytes(struct.pack("<4I", 0x4D455348, 0, 1, 1) + _compressed(faces.tobytes(), width)
                                        + _compressed(nodes.tobytes(), width))
    s = pt.Scene.load(tmp_path / "ref.json")
    assert s.counts() == (0, 1, 1, 0)
    a = packed(s)
    assert len(a["shapes"]) == 1 and a["shapes"][0]["Type"] == 2          # SHAPE_TYPE_SPHERE
    assert a["globals"][0]["SkyboxBrightness"] == 2.0
    assert len(a["mesh_nodes"]) == 1 and len(a["mesh_faces"]) == 1      # mesh packed, no instance
    assert a["cameras"][0]["Model"] == 0
    s.close()


def test_load_errors(pt, tmp_path):
    with pytest.raises(RuntimeError, match="cannot open"):
        pt.Scene.load(tmp_path / "missing.json")
    (tmp_path / "bad.json").write_text('{"Root": [1, 2,, 3]}')
    with pytest.raises(RuntimeError, match="scene JSON"):
        pt.Scene.load(tmp_path / "bad.json")
    (tmp_path / "t.json").write_text('{"Textures": [{"Name": "Gone", "Type": 0, "EnableNearestFiltering": false}]}')
    with pytest.raises(RuntimeError, match="texture"):
        pt.Scene.load(tmp_path / "t.json")
