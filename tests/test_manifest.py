"""manifest.json (optional part): s3imph_write_manifest / verify / sha256_file
against the reference's manifest tests (/root/reference/pkg/format/manifest_test.go:10-160)
and Go's encoding/json layout.  Host-only, no GPU.  hashlib is the SHA-256 checker here."""
import hashlib
import json
import os
import re

import pytest

import oracle as O
import s3imph

RFC3339NANO = re.compile(r"^\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d(\.\d*[1-9])?Z$")


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 65, 119, 120, 4099, (4 << 20) + 17])
def test_sha256_matches_hashlib(tmp_path, n):
    """Both compression paths (x86 SHA extensions and the portable loop) == hashlib, around
    the padding boundaries (55/56/64 B) and the 4 MiB read chunk."""
    data = os.urandom(n)
    p = tmp_path / "x.bin"
    p.write_bytes(data)
    want = hashlib.sha256(data).hexdigest()
    assert s3imph.sha256_file(str(p)) == want
    assert s3imph.sha256_file(str(p), portable=True) == want


def test_checksum_deterministic_and_data_dependent(tmp_path):
    """TestChecksumFile (manifest_test.go:103-141)."""
    p = tmp_path / "test.bin"
    p.write_bytes(b"hello world")
    c1, c2 = s3imph.sha256_file(str(p)), s3imph.sha256_file(str(p))
    assert c1 == c2 == hashlib.sha256(b"hello world").hexdigest()
    p.write_bytes(b"different")
    assert s3imph.sha256_file(str(p)) != c1


def test_write_and_read_manifest(tmp_path):
    """TestWriteAndReadManifest (manifest_test.go:10-61): listed files only, sizes and
    checksums, version / node_count / max_depth."""
    files = {"subtree_end.u64": b"test data 1", "depth.u32": b"test data 2", "unrelated.txt": b"x"}
    for name, data in files.items():
        (tmp_path / name).write_bytes(data)
    s3imph.write_manifest(str(tmp_path), 100, 5)
    m = s3imph.read_manifest(str(tmp_path))
    assert m["version"] == 1 and m["node_count"] == 100 and m["max_depth"] == 5
    assert RFC3339NANO.match(m["created_at"]), m["created_at"]
    assert set(m["files"]) == {"subtree_end.u64", "depth.u32"}
    for name in m["files"]:
        assert m["files"][name] == {"size": len(files[name]), "checksum": hashlib.sha256(files[name]).hexdigest()}


def test_manifest_text_is_go_marshal_indent(tmp_path):
    """The bytes equal json.MarshalIndent(manifest, "", "  "): struct field order, sorted
    map keys, ": " / "," separators, no trailing newline (Python's json.dumps(indent=2)
    renders the same layout); an empty file map is {}."""
    s3imph.write_manifest(str(tmp_path), 0, 0)
    text = (tmp_path / "manifest.json").read_text()
    m = json.loads(text)
    assert m["files"] == {}
    assert text == json.dumps({"version": 1, "created_at": m["created_at"], "node_count": 0, "max_depth": 0,
                               "files": {}}, indent=2)
    for name in ["mph.bin", "depth.u32", "prefix_blob.bin"]:
        (tmp_path / name).write_bytes(name.encode() * 3)
    s3imph.write_manifest(str(tmp_path), 7, 2)
    text = (tmp_path / "manifest.json").read_text()
    m = json.loads(text)
    files = {k: {"size": 3 * len(k), "checksum": hashlib.sha256(k.encode() * 3).hexdigest()}
             for k in sorted(["mph.bin", "depth.u32", "prefix_blob.bin"])}
    assert text == json.dumps({"version": 1, "created_at": m["created_at"], "node_count": 7, "max_depth": 2,
                               "files": files}, indent=2)


def test_verify_manifest_detects_corruption(tmp_path):
    """TestVerifyManifest (manifest_test.go:63-101), plus a size change and a missing file."""
    p = tmp_path / "subtree_end.u64"
    p.write_bytes(b"test data for verification")
    s3imph.write_manifest(str(tmp_path), 50, 3)
    s3imph.verify_manifest(str(tmp_path))
    p.write_bytes(b"test data for verificatioN")  # same size, other bytes
    with pytest.raises(s3imph.MPHFError, match="checksum mismatch") as e:
        s3imph.verify_manifest(str(tmp_path))
    assert e.value.status == s3imph.ERR_FORMAT
    p.write_bytes(b"corrupted data")
    with pytest.raises(s3imph.MPHFError, match=r"size mismatch \(got 14, want 26\)"):
        s3imph.verify_manifest(str(tmp_path))
    p.unlink()
    with pytest.raises(s3imph.MPHFError) as e:
        s3imph.verify_manifest(str(tmp_path))
    assert e.value.status == s3imph.ERR_IO


def test_manifest_over_index_files(tmp_path, oracle_lib):
    """The five MPHF files write_index_files emits, checksummed as the reference's
    Finalize would (indexbuild.go:429-432); verify passes, and a manifest written by the
    reference's layout (another created_at, compact spacing) is read the same way."""
    keys = [b"", b"a/", b"a/b/", b"b/", b"c/"]
    blob, offs = O.keys_to_blob(keys)
    st, fp, pos, mph = oracle_lib.build(blob, offs)
    s3imph.write_index_files(str(tmp_path), mph, fp, pos, blob, offs)
    s3imph.write_manifest(str(tmp_path), len(keys), 2)
    m = s3imph.read_manifest(str(tmp_path))
    assert sorted(m["files"]) == sorted(["mph.bin", "mph_fp.u64", "mph_pos.u64", "prefix_blob.bin",
                                         "prefix_offsets.u64"])
    for name, fi in m["files"].items():
        data = (tmp_path / name).read_bytes()
        assert fi == {"size": len(data), "checksum": hashlib.sha256(data).hexdigest()}
    s3imph.verify_manifest(str(tmp_path))
    m["created_at"] = "2025-01-02T03:04:05.5Z"
    (tmp_path / "manifest.json").write_text(json.dumps(m, separators=(",", ":")))
    s3imph.verify_manifest(str(tmp_path))
