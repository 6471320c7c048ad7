#!/usr/bin/env python3
"""Loader edge cases (LoadSceneJSON / LoadMesh, Raytracer.cpp:589-779) pinned by
the REFERENCE ITSELF: each case is a scene (and mesh) file written under
tests/golden/loader/Assets/, loaded by the reference binary (oracle/_ref,
built from /root/reference) which records its LoadSceneJSON status and, when
the load succeeds, the sha256 of a tiny render (8x6, depth 1, AO off).
Build container only:  make -C oracle ref && python tests/golden/make_loader_goldens.py

Cases where the reference's behaviour is undefined (a missing key read from a
const nlohmann::json, an unknown light type leaving lightType uninitialised)
are not generated here; tests/test_loader.py pins the repository's defined
choice for those (RT_FAILURE) separately."""
import hashlib
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "loader")
ASSETS = os.path.join(OUT, "Assets")
REF = os.path.join(REPO, "oracle", "_ref", "rt_ref_param")

SPHERE_MESH = '{"data": [{"type": "sphere", "radius": 1}]}'
FLOOR_MESH = open(os.path.join(HERE, "Assets", "floor.json")).read()
TWO_TRI_TYPE_FIRST_ONLY = json.dumps({"data": [
    {"type": "polygon", "v0": {"v": [-2, 0, -2], "n": [0, 1, 0], "t": [0, 0]},
     "v1": {"v": [2, 0, -2], "n": [0, 1, 0], "t": [1, 0]}, "v2": {"v": [0, 0, 2], "n": [0, 1, 0], "t": [0, 1]}},
    {"v0": {"v": [-2, 1, -2], "n": [0, 0, 1], "t": [0, 0]},
     "v1": {"v": [2, 1, -2], "n": [0, 0, 1], "t": [1, 0]}, "v2": {"v": [0, 3, -2], "n": [0, 0, 1], "t": [0, 1]}}]})


def scene(shapes_text=None, lights_text=None, camera_text=None, extra=""):
    shapes_text = shapes_text if shapes_text is not None else (
        '[{"id": "s1", "geometry": "lsphere", "material": {"Cs": [1, 0.2, 0.2], "Ka": 0.4, "Kd": 0.7, '
        '"Ks": 0.3, "Kt": 0, "n": 20}, "transforms": [{"S": [1, 1, 1]}, {"T": [0, 1, 0]}]},'
        ' {"id": "f", "geometry": "lfloor", "material": {"Cs": [0.8, 0.8, 0.8], "Ka": 0.3, "Kd": 0.6, '
        '"Ks": 0.1, "Kt": 0, "n": 5}, "transforms": [{"Ry": 10}]}]')
    lights_text = lights_text if lights_text is not None else (
        '[{"id": "a", "type": "ambient", "color": [1, 1, 1], "intensity": 0.2},'
        ' {"id": "d", "type": "directional", "color": [1, 1, 1], "intensity": 0.8, "from": [1, 4, 2], "to": [0, 0, 0]}]')
    camera_text = camera_text if camera_text is not None else (
        '{"from": [0, 2, 6], "to": [0, 1, 0], "bounds": [0.1, 100, 1, -1, 1, -1], "resolution": [8, 6]}')
    return '{"scene": {"shapes": %s, "camera": %s, "lights": %s%s}}' % (shapes_text, camera_text, lights_text, extra)


BASE = scene()
CASES = {
    "base": BASE,
    "number_malformed": BASE.replace('"Ka": 0.4', '"Ka": 0.4.5'),
    "number_leading_zero": BASE.replace('"Ka": 0.4', '"Ka": 04'),
    "number_trailing_dot": BASE.replace('"Ka": 0.4', '"Ka": 4.'),
    "number_leading_dot": BASE.replace('"Ka": 0.4', '"Ka": .4'),
    "number_plus": BASE.replace('"Ka": 0.4', '"Ka": +0.4'),
    "number_exponent": BASE.replace('"Ka": 0.4', '"Ka": 4E-1'),
    "number_integer": BASE.replace('"Kd": 0.7', '"Kd": 1'),
    "number_huge": BASE.replace('"n": 20', '"n": 1e39'),
    "number_many_digits": BASE.replace('"Ka": 0.4', '"Ka": 0.40000000000000002220446049250313080847263336181640625'),
    "trailing_comma": BASE.replace('"n": 20}', '"n": 20,}'),
    "comment": BASE.replace('"transforms"', '/* c */ "transforms"'),
    "string_for_number": BASE.replace('"Ka": 0.4', '"Ka": "0.4"'),
    "null_for_number": BASE.replace('"Ka": 0.4', '"Ka": null'),
    "bool_for_number": BASE.replace('"Ka": 0.4', '"Ka": true'),
    "notes_string": BASE.replace('"id": "s1",', '"id": "s1", "notes": "a red ball",'),
    "notes_number": BASE.replace('"id": "s1",', '"id": "s1", "notes": 5,'),
    "id_number": BASE.replace('"id": "s1"', '"id": 1'),
    "rotation_string": BASE.replace('{"Ry": 10}', '{"Ry": "10"}'),
    "scale_not_array": BASE.replace('{"S": [1, 1, 1]}', '{"S": 2}'),
    "transforms_override": BASE.replace('[{"S": [1, 1, 1]}, {"T": [0, 1, 0]}]',
                                        '[{"T": [5, 5, 5]}, {"S": [1, 1, 1]}, {"T": [0, 1, 0]}]'),
    "duplicate_key": BASE.replace('"Ka": 0.4', '"Ka": 0.9, "Ka": 0.4'),
    "unicode_escape_id": BASE.replace('"id": "s1"', '"id": "s\\u0031\\u00e9"'),
    "bom": "﻿" + BASE,
    "crlf_tabs": BASE.replace(", ", ",\r\n\t"),
    "no_shapes_key": scene(extra="").replace('"shapes": ', '"shapez": '),
    "empty_shapes": scene(shapes_text="[]"),
    "no_lights": scene(lights_text="[]"),
    "no_scene_key": '{"notscene": {}}',
    "type_on_first_item_only": scene(shapes_text='[{"id": "m", "geometry": "ltwo", "material": {"Cs": [0.2, 0.9, 0.2], '
                                     '"Ka": 0.5, "Kd": 0.5, "Ks": 0.2, "Kt": 0, "n": 10}, "transforms": []}]'),
    "mesh_malformed": scene(shapes_text='[{"id": "m", "geometry": "lbad", "material": {"Cs": [1, 1, 1], '
                            '"Ka": 0.5, "Kd": 0.5, "Ks": 0, "Kt": 0, "n": 2}, "transforms": []}]'),
    "mesh_missing": scene(shapes_text='[{"id": "m", "geometry": "lnothere", "material": {"Cs": [1, 1, 1], '
                          '"Ka": 0.5, "Kd": 0.5, "Ks": 0, "Kt": 0, "n": 2}, "transforms": []}]'),
    "mesh_plane_type": scene(shapes_text='[{"id": "p", "geometry": "lplane", "material": {"Cs": [1, 1, 1], '
                             '"Ka": 0.5, "Kd": 0.5, "Ks": 0, "Kt": 0, "n": 2}, "transforms": []},'
                             '{"id": "s", "geometry": "lsphere", "material": {"Cs": [1, 1, 1], '
                             '"Ka": 0.5, "Kd": 0.5, "Ks": 0, "Kt": 0, "n": 2}, "transforms": []}]'),
    "truncated": BASE[:len(BASE) // 2],
    "empty_file": "",
    "null_document": "null",
    "array_document": "[]",
    "number_document": "5",
    "scene_null": '{"scene": null}',
}
MESHES = {
    "lsphere.json": SPHERE_MESH,
    "lfloor.json": FLOOR_MESH,
    "ltwo.json": TWO_TRI_TYPE_FIRST_ONLY,
    "lbad.json": '{"data": [{"type": "polygon", "v0": {"v": [0, 0, 0.1.2]}}]}',
    "lplane.json": '{"data": [{"type": "plane", "width": 4}]}',
}


def main():
    os.makedirs(ASSETS, exist_ok=True)
    for name, text in MESHES.items():
        open(os.path.join(ASSETS, name), "w", encoding="utf-8", newline="").write(text)
    results = []
    for name, text in CASES.items():
        fn = "case_%s.json" % name
        open(os.path.join(ASSETS, fn), "w", encoding="utf-8", newline="").write(text)
        out = "/tmp/loader_%s.ppm" % name
        if os.path.exists(out):
            os.remove(out)
        p = subprocess.run([REF, OUT, fn, "8", "6", "1", out, "128", "1"], capture_output=True, text=True,
                           timeout=120)
        loaded = "LoadSceneJSON failed" not in p.stderr and p.returncode in (0,)
        rec = {"name": name, "file": fn, "reference_exit": p.returncode, "load_ok": loaded}
        if "LoadSceneJSON failed" in p.stderr:
            rec["load_status"] = int(p.stderr.split("LoadSceneJSON failed:")[1].split()[0])
        if loaded and os.path.exists(out):
            rec["ppm_sha256"] = hashlib.sha256(open(out, "rb").read()).hexdigest()
        results.append(rec)
        print(name, rec)
    json.dump({"generator": "tests/golden/make_loader_goldens.py", "reference_binary": "rt_ref_param",
               "render": {"width": 8, "height": 6, "depth": 1, "ao_enabled": False}, "cases": results},
              open(os.path.join(OUT, "manifest.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
