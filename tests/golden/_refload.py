"""Import the read-only reference (/root/reference) for FIXTURE GENERATION ONLY.

Runs only in the build container (the reference never travels to the GPU box).
Recipe follows SURVEY.md §8(c): vendored diffusers 0.30 on sys.path, the three
transformers-5.x constants diffusers expects
(diffusers/pipelines/pipeline_loading_utils.py:48-50), stubs for `av` /
`torchvision` (only used by video_io / restore_res, never by `forward`), and the
depth pipeline modules loaded by file path so that rollingdepth/__init__.py
(which imports the IC-Light experiments) is never executed.
"""
import importlib.util
import os
import sys
import types

REF = "/root/reference"


def load_reference():
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    src = os.path.join(REF, "diffusers", "src")
    if src not in sys.path:
        sys.path.insert(0, src)
    import transformers.utils as tu

    for name, val in (
        ("FLAX_WEIGHTS_NAME", "flax_model.msgpack"),
        ("SAFE_WEIGHTS_NAME", "model.safetensors"),
        ("WEIGHTS_NAME", "pytorch_model.bin"),
    ):
        if not hasattr(tu, name):
            setattr(tu, name, val)
    import diffusers  # noqa: F401  (before the stubs: diffusers probes find_spec)

    # stubs for modules absent from the image and unused by forward()
    if "av" not in sys.modules:
        sys.modules["av"] = types.ModuleType("av")
    if "torchvision" not in sys.modules:
        tv = types.ModuleType("torchvision")
        tvt = types.ModuleType("torchvision.transforms")
        tvf = types.ModuleType("torchvision.transforms.functional")

        class InterpolationMode:  # noqa: D401 - stub
            BILINEAR = "bilinear"

        tvt.InterpolationMode = InterpolationMode
        tvf.resize = lambda *a, **k: (_ for _ in ()).throw(RuntimeError("stub"))
        tvt.functional = tvf
        tv.transforms = tvt
        sys.modules["torchvision"] = tv
        sys.modules["torchvision.transforms"] = tvt
        sys.modules["torchvision.transforms.functional"] = tvf

    if "rollingdepth" not in sys.modules:
        pkg = types.ModuleType("rollingdepth")
        pkg.__path__ = [os.path.join(REF, "rollingdepth")]
        sys.modules["rollingdepth"] = pkg
        for mod in ("video_io", "depth_aligner", "rollingdepth_pipeline"):
            full = f"rollingdepth.{mod}"
            spec = importlib.util.spec_from_file_location(
                full, os.path.join(REF, "rollingdepth", mod + ".py")
            )
            m = importlib.util.module_from_spec(spec)
            sys.modules[full] = m
            spec.loader.exec_module(m)
    return sys.modules["rollingdepth.rollingdepth_pipeline"], sys.modules["rollingdepth.depth_aligner"]
