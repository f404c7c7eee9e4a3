"""The FFmpeg-side glue (integration/vp9_hip.c: the FFHWAccel; integration/hwcontext_hip.c:
the HWContextType) type-checks against the FFmpeg 8.0 declarations it binds.

FFmpeg's headers need the configure-generated config.h / avconfig.h, so the glue compiles
(gcc -fsyntax-only -Wall -Werror) against tests/glue/ffmpeg_decls.h, a restatement of exactly
the declarations it uses, through shim headers named like FFmpeg's. The restatement is
pinned to the reference: every restated line carries a marker naming the reference header
(and the struct / enum it belongs to), and test_restated_declarations_match_reference finds
each normalised line there (skipped where /root/reference is absent). A deliberately wrong
callback signature must fail the check.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
DECLS = os.path.join(ROOT, "tests", "glue", "ffmpeg_decls.h")
GLUE = [os.path.join(ROOT, "integration", "vp9_hip.c"), os.path.join(ROOT, "integration", "hwcontext_hip.c")]

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")


def _gcc(src):
    g = os.path.join(ROOT, "tests", "glue")
    cmd = ["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Werror", "-Wno-unused-function", "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", "-I" + g, "-I" + os.path.join(g, "inc"), "-I" + os.path.join(g, "inc", "libavutil"),
           "-I" + os.path.join(ROOT, "include"), src]
    return subprocess.run(cmd, capture_output=True, text=True)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"), reason="HIP headers absent")
@pytest.mark.parametrize("src", GLUE, ids=lambda p: os.path.basename(p))
def test_glue_typechecks(src):
    r = _gcc(src)
    assert r.returncode == 0, r.stderr


@pytest.mark.skipif(not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"), reason="HIP headers absent")
@pytest.mark.parametrize("src,old,new", [
    # an FFHWAccel callback with the wrong parameter list
    ("vp9_hip.c", "static int vp9_hip_end_frame(AVCodecContext *avctx)", "static int vp9_hip_end_frame(AVCodecContext *avctx, int x)"),
    # start_frame without the buf_ref parameter FFmpeg 8.0 passes
    ("vp9_hip.c", "static int vp9_hip_start_frame(AVCodecContext *avctx, const AVBufferRef *buf_ref, const uint8_t *buf, uint32_t size)",
     "static int vp9_hip_start_frame(AVCodecContext *avctx, const uint8_t *buf, uint32_t size)"),
    # a HWContextType transfer callback with a non-const source
    ("hwcontext_hip.c", "static int hip_transfer_data_from(AVHWFramesContext *ctx, AVFrame *dst, const AVFrame *src)",
     "static int hip_transfer_data_from(AVHWFramesContext *ctx, AVFrame *dst, AVFrame *src)"),
])
def test_wrong_signature_fails(tmp_path, src, old, new):
    text = open(os.path.join(ROOT, "integration", src)).read()
    assert old in text
    bad = tmp_path / src
    bad.write_text(text.replace(old, new))
    if src == "hwcontext_hip.c":                  # its own header next to it, as in the tree
        shutil.copy(os.path.join(ROOT, "integration", "hwcontext_hip.h"), tmp_path / "hwcontext_hip.h")
    r = _gcc(str(bad))
    assert r.returncode != 0 and "error" in r.stderr


def _norm(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    s = re.sub(r"//[^\n]*", " ", s)
    s = s.replace("\\\n", " ")
    s = re.sub(r"#\s*define", "#define", s)
    s = re.sub(r"\s+", " ", s)
    s = re.sub(r"\s*([(){}\[\];,*=<>&|!?:~^+\-])\s*", r"\1", s)
    return s.strip()


def _body(text, name):
    """The {...} body of struct / union / enum `name` (typedef'd or tagged) in normalised text."""
    for pat in (r"(?:struct|union|enum) %s\{" % re.escape(name), r"typedef (?:struct|union|enum)\{"):
        for m in re.finditer(pat, text):
            depth, i = 0, m.end() - 1
            for j in range(i, len(text)):
                depth += text[j] == "{"
                depth -= text[j] == "}"
                if depth == 0:
                    body = text[i:j + 1]
                    tail = text[j + 1:j + 1 + len(name) + 2]
                    if pat.startswith("typedef") and not tail.startswith(name):
                        break
                    return body
    return None


def _check_decls(decls):
    """(checked, mismatches) of the restated lines of `decls` against the reference."""
    checked, bad = 0, []
    cache = {}
    for ln, line in enumerate(open(decls), 1):
        m = re.search(r"/\*@ (\S+)(?: in (\w+))? \*/\s*$", line)
        if not m:
            continue
        decl, path, scope = _norm(line[:m.start()]), m.group(1), m.group(2)
        if path not in cache:
            cache[path] = _norm(open(os.path.join(REF, path), errors="replace").read())
        text = cache[path]
        if scope:
            text = _body(text, scope) or ""
        # a function prototype: up to the parameter list (the reference adds attributes)
        if decl.endswith(");") and not decl.startswith(("int(", "void(", "AVBufferRef*(")) and "(*" not in decl.split("(")[0]:
            decl = decl[:-1]
        if decl.endswith("{") and not scope:
            decl = decl[:-1].rstrip()
        checked += 1
        if decl not in text:
            bad.append((ln, path, scope, decl))
    return checked, bad


@pytest.mark.skipif(not os.path.isdir(REF), reason="/root/reference absent")
def test_restated_declarations_match_reference():
    checked, bad = _check_decls(DECLS)
    assert checked > 150
    assert not bad, "restated declarations not found in the reference:\n" + "\n".join(map(str, bad))


@pytest.mark.skipif(not os.path.isdir(REF), reason="/root/reference absent")
@pytest.mark.parametrize("old,new", [
    ("    int (*end_frame)(AVCodecContext *avctx);", "    int (*end_frame)(AVCodecContext *avctx, int x);"),
    ("    AVBufferPool *pool_internal;", "    AVBufferRef *pool_internal;"),
    ("#define CUR_FRAME 0", "#define CUR_FRAME 1"),
])
def test_restatement_check_catches_drift(tmp_path, old, new):
    text = open(DECLS).read()
    assert old in text
    p = tmp_path / "decls.h"
    p.write_text(text.replace(old, new, 1))
    _, bad = _check_decls(str(p))
    assert len(bad) == 1
