"""Hash of the sources librtpt.so is built from (csrc/*, include/*).

tools/profile.sh records it in every rocprof summary and bench.py only uses a
committed summary (profiles/pmc_summary.json) whose hash matches the tree:
a counter total measured on another kernel version is never reported.
Standalone (no library load) so the profiler tooling can import it.
"""
import hashlib
import os

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def have_sources() -> bool:
    """Whether the library's source directories are present (an installed
    package may ship librtpt.so without them)."""
    return all(os.path.isdir(os.path.join(_ROOT, sub)) for sub in ("gpuraytracer_amd/csrc", "include"))


def kernel_source_sha() -> str:
    h = hashlib.sha256()
    for sub in ("gpuraytracer_amd/csrc", "include"):
        d = os.path.join(_ROOT, sub)
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".hpp", ".h", ".cpp")):
                h.update(f.encode())
                h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


if __name__ == "__main__":  # the Makefile compiles this into librtpt.so (rt_build_sha)
    print(kernel_source_sha())
