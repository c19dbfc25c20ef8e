"""The C++ host mirror of liboxen `util::hasher` (oxen_amd/host) and its native test program
(tests/native/test_hasher.cpp: the reference's hasher.rs tests, known answers, error behaviour)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def native(built_lib):
    from oxen_amd import build

    build.build_host()
    return build.NATIVE_TEST


def test_mirror_builds_and_exports_the_hasher_api(native):
    from oxen_amd import build

    out = subprocess.run(["nm", "-DC", "--defined-only", build.HOST_LIB], capture_output=True, text=True, check=True).stdout
    for name in ["liboxen::util::hasher::hash_buffer_128bit", "liboxen::util::hasher::hash_file_contents",
                 "liboxen::util::hasher::get_hash_given_metadata", "liboxen::util::hasher::get_combined_hash",
                 "liboxen::util::hasher::get_metadata_hash", "liboxen::util::hasher::Xxh3::digest128",
                 "liboxen::util::hasher::hash_files", "liboxen::MerkleHash::from_str",
                 "liboxen::util::hasher::ReaderPool::hash_files",
                 "liboxen::util::fs::classify_modified_batch", "liboxen::util::fs::AtomicFile::stream",
                 "liboxen::storage::LocalVersionStore::store_version_from_reader",
                 "liboxen::storage::LocalVersionStore::store_versions"]:
        assert name in out, name
    assert os.access(native, os.X_OK)


def test_mirror_refuses_without_a_gpu(native):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([native, GOLDEN], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "oxh_ctx_create" in r.stderr  # no CPU fallback


@pytest.mark.gpu
def test_native_hasher_mirror_on_gpu(cuda, native):
    r = subprocess.run([native, GOLDEN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout
