#!/usr/bin/env python3
"""Generate the committed golden fixtures from the REFERENCE ITSELF (test infrastructure).

Runs oracle/_ref/rt_ref_strict and oracle/_ref/rt_ref_fast -- the unmodified reference sources
(/root/reference/cpu/src/*.c) linked with oracle/ref_harness.c, built by oracle/Makefile -- on the
scenes in assets/*.tar.gz and stores:

  <scene>_<W>x<H>_<flavour>.npz   full int32 hit / f32 t / f32 rgb[H,W,3] arrays (small frames)
  <scene>_1080p_<flavour>_sample.npz  every 97th pixel of the 1920x1080 frame (idx, hit, t, rgb)
  golden.json                      md5 of full-resolution frames and of the BVH dumps, plus the
                                   SURVEY §8c values they must equal

  stress (round 2): the high-triangle-count workloads -- the sportscar stand-in (514k-triangle car, the
  real sportscar .mtl), dragon871k (Stanford-dragon triangle count) and random mode at 1M triangles
  (main.c:115-131) -- at 96x54 (full arrays), 320x180 (md5), and for the 1080p frames of dragon,
  dragon871k and sportscar every 97th pixel, the full frame's md5 and the reference's ray counts.

Frame binary layout (ref_harness.c): int32 hit[N] | f32 t[N] | f32 rgb[3N], row-major idx = y*W + x.
Only needed in the build container (where /root/reference exists); the fixtures are committed.
  configs (round 3): two_cars at 3840x2160 and dragon at 640x360 (BASELINE configs 4 and 1).

usage: make_golden.py [all | cars | standin | stress | configs ...]  (sections update golden.json in place)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from tests.scenes import scene_paths  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref")


def run(binary, *args):
    subprocess.run([os.path.join(REF, binary)] + [str(a) for a in args], check=True,
                   stdout=subprocess.DEVNULL)


def frame(path, W, H):
    raw = open(path, "rb").read()
    N = W * H
    hit = np.frombuffer(raw[: 4 * N], np.int32).reshape(H, W)
    t = np.frombuffer(raw[4 * N: 8 * N], np.float32).reshape(H, W)
    rgb = np.frombuffer(raw[8 * N:], np.float32).reshape(H, W, 3)
    return raw, hit, t, rgb


def counts(scene_files, W, H, tmp):
    """the reference's own ray counts (rt_ref_count: linker-wrapped traversal calls)"""
    p = os.path.join(tmp, "c.bin")
    r = subprocess.run([os.path.join(REF, "rt_ref_count"), "render", *scene_files, str(W), str(H),
                        str(os.cpu_count() or 8), p], check=True, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                       text=True)
    line = [l for l in r.stderr.splitlines() if l.startswith("COUNTS")][-1]
    kv = dict(x.split("=") for x in line.split()[1:])
    closest = int(kv["trav"]) - W * H
    return {"closest": closest, "shadow": int(kv["light"]), "total": closest + int(kv["light"])}


def standin(out, tmp, names):
    out.setdefault("standin", {})
    for scene in names:
        obj, mtl, lts = scene_paths(scene)
        ent = {"obj_md5": hashlib.md5(open(obj, "rb").read()).hexdigest()}
        for (W, H) in ((96, 54), (320, 180)):
            p = os.path.join(tmp, f"{scene}_{W}x{H}.bin")
            run("rt_ref_strict", "render", obj, mtl, lts, W, H, os.cpu_count() or 8, p)
            raw, hit, t, rgb = frame(p, W, H)
            ent[f"{W}x{H}_md5"] = hashlib.md5(raw).hexdigest()
            if W == 96:
                np.savez_compressed(os.path.join(HERE, f"{scene}_{W}x{H}_strict.npz"), hit=hit, t=t, rgb=rgb)
        p = os.path.join(tmp, f"{scene}.bvh")
        run("rt_ref_strict", "bvh", obj, mtl, p)
        raw = open(p, "rb").read()
        ent["bvh_h3_md5"] = hashlib.md5(raw).hexdigest()
        ent["bvh_h3_nodes"] = int(np.frombuffer(raw[:4], np.int32)[0])
        out["standin"][scene] = ent


def stress(out, tmp):
    standin(out, tmp, ("sportscar", "dragon871k"))
    out.setdefault("rays", {})
    for scene in ("dragon", "dragon871k", "sportscar"):
        W, H = 1920, 1080
        p = os.path.join(tmp, f"{scene}_1080p.bin")
        run("rt_ref_strict", "render", *scene_paths(scene), W, H, os.cpu_count() or 8, p)
        raw, hit, t, rgb = frame(p, W, H)
        out["standin"][scene]["1920x1080_md5"] = hashlib.md5(raw).hexdigest()
        idx = np.arange(0, W * H, 97)
        np.savez_compressed(os.path.join(HERE, f"{scene}_1080p_strict_sample.npz"), idx=idx,
                            hit=hit.reshape(-1)[idx], t=t.reshape(-1)[idx], rgb=rgb.reshape(-1, 3)[idx])
        os.remove(p)
        out["rays"][f"{scene}_{W}x{H}"] = counts(scene_paths(scene), W, H, tmp)
    # random-triangle mode at 1M triangles (SURVEY §8d's BVH stress): primary rays only (kr = 0, no lights)
    p = os.path.join(tmp, "random1m.bin")
    run("rt_ref_strict", "random", 1000000, 96, 54, os.cpu_count() or 8, p)
    raw, hit, t, rgb = frame(p, 96, 54)
    np.savez_compressed(os.path.join(HERE, "random1m_96x54_strict.npz"), hit=hit, t=t, rgb=rgb)
    out["frames"]["random1m_96x54_strict"] = {"md5": hashlib.md5(raw).hexdigest(), "W": 96, "H": 54}
    p = os.path.join(tmp, "random1m.bvh")
    run("rt_ref_strict", "bvhrand", 1000000, p)
    raw = open(p, "rb").read()
    out["bvh"]["random1m_h3"] = {"md5": hashlib.md5(raw).hexdigest(), "nodes": int(np.frombuffer(raw[:4], np.int32)[0])}


def configs(out, tmp):
    """round 3: the two BASELINE configurations no fixture covered yet, at the sizes BASELINE.json names --
    two_cars at 3840x2160 (every 97th pixel, the frame's md5, rt_ref_count's rays) and dragon at 640x360
    (cpu/src/main.c's own WIDTH x HEIGHT: every 7th pixel, the frame's md5, rays)"""
    out.setdefault("rays", {})
    for scene, W, H, step, tag in (("two_cars", 3840, 2160, 97, "2160p"), ("dragon", 640, 360, 7, "360p")):
        p = os.path.join(tmp, f"{scene}_{tag}.bin")
        run("rt_ref_strict", "render", *scene_paths(scene), W, H, os.cpu_count() or 8, p)
        raw, hit, t, rgb = frame(p, W, H)
        out["standin"][scene][f"{W}x{H}_md5"] = hashlib.md5(raw).hexdigest()
        idx = np.arange(0, W * H, step)
        np.savez_compressed(os.path.join(HERE, f"{scene}_{tag}_strict_sample.npz"), idx=idx,
                            hit=hit.reshape(-1)[idx], t=t.reshape(-1)[idx], rgb=rgb.reshape(-1, 3)[idx])
        os.remove(p)
        out["rays"][f"{scene}_{W}x{H}"] = counts(scene_paths(scene), W, H, tmp)


def main(sections):
    gpath = os.path.join(HERE, "golden.json")
    out = json.load(open(gpath)) if os.path.exists(gpath) and "all" not in sections else {}
    out.setdefault("generator", "tests/golden/make_golden.py")
    out.setdefault("frames", {})
    out.setdefault("bvh", {})
    tmp = tempfile.mkdtemp()
    if "stress" in sections:
        stress(out, tmp)
    if "configs" in sections:
        configs(out, tmp)
    if "standin" in sections or "all" in sections:
        standin(out, tmp, ("dragon", "sportscar", "two_cars"))
    if "cars" not in sections and "all" not in sections:
        with open(gpath, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
        return
    for scene in ("car_boxed", "car_only"):
        obj, mtl, lts = scene_paths(scene)
        for flav, binary in (("strict", "rt_ref_strict"), ("fast", "rt_ref_fast")):
            for (W, H) in ((160, 90), (64, 36), (640, 360), (1920, 1080)):
                p = os.path.join(tmp, f"{scene}_{W}x{H}_{flav}.bin")
                run(binary, "render", obj, mtl, lts, W, H, os.cpu_count() or 8, p)
                raw, hit, t, rgb = frame(p, W, H)
                key = f"{scene}_{W}x{H}_{flav}"
                out["frames"][key] = {"md5": hashlib.md5(raw).hexdigest(), "W": W, "H": H,
                                      "primary_hits": int((hit >= 0).sum())}
                if W * H <= 160 * 90:
                    np.savez_compressed(os.path.join(HERE, key + ".npz"), hit=hit, t=t, rgb=rgb)
                if W == 1920:
                    idx = np.arange(0, W * H, 97)
                    np.savez_compressed(os.path.join(HERE, f"{scene}_1080p_{flav}_sample.npz"), idx=idx,
                                        hit=hit.reshape(-1)[idx], t=t.reshape(-1)[idx],
                                        rgb=rgb.reshape(-1, 3)[idx])
                os.remove(p)
        p = os.path.join(tmp, f"{scene}.bvh")
        run("rt_ref_strict", "bvh", obj, mtl, p)
        raw = open(p, "rb").read()
        out["bvh"][f"{scene}_h3"] = {"md5": hashlib.md5(raw).hexdigest(),
                                     "nodes": int(np.frombuffer(raw[:4], np.int32)[0])}
    # random-triangle mode (cpu/src/main.c:115-131): 10,000 tris, 160x90, no lights
    p = os.path.join(tmp, "random.bin")
    run("rt_ref_strict", "random", 10000, 160, 90, 8, p)
    raw, hit, t, rgb = frame(p, 160, 90)
    np.savez_compressed(os.path.join(HERE, "random10k_160x90_strict.npz"), hit=hit, t=t, rgb=rgb)
    out["frames"]["random10k_160x90_strict"] = {"md5": hashlib.md5(raw).hexdigest(), "W": 160, "H": 90}
    p = os.path.join(tmp, "random.bvh")
    run("rt_ref_strict", "bvhrand", 10000, p)
    raw = open(p, "rb").read()
    out["bvh"]["random10k_h3"] = {"md5": hashlib.md5(raw).hexdigest(),
                                  "nodes": int(np.frombuffer(raw[:4], np.int32)[0])}
    # ray counts from the reference itself (rt_ref_count: linker-wrapped traversal calls)
    out.setdefault("rays", {})
    for scene in ("car_boxed", "car_only"):
        for (W, H) in ((160, 90), (1920, 1080)):
            out["rays"][f"{scene}_{W}x{H}"] = counts(scene_paths(scene), W, H, tmp)
    # values SURVEY §8c / Appendix A recorded independently during the survey
    out["survey"] = {
        "car_boxed_1920x1080_strict": "6caa907524126a25bf7bdce0610a6586",
        "car_boxed_1920x1080_fast_survey_host": "7afffe2defeeb4c31e05d75175266c87",
        "car_only_1920x1080_strict": "3fadf174f30556ebe62834afc40124f8",
        "car_boxed_640x360_strict": "5f19941c9cc7817627e77c9ceb26ef88",
        "bvh_car_boxed_h3": "dbba8cd40af19553fe21f622f18bd4b9",
        "bvh_car_boxed_h6": "359ad63d3f0b8d4647222514e7867f0d",
        "bvh_car_only_h3": "39ce27cf822e6b20631cdeea4d81f6de",
        "car_boxed_1080p_rays": 13247875,
        "car_only_1080p_rays_survey_note": "SURVEY says 2978529; the reference counted by rt_ref_count gives 2978527",
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1:] or ["all"])
