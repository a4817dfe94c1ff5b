"""bench.py's roofline bookkeeping (CPU): every kernel the encoder launches is priced against the MFMA
ceiling of the arithmetic it runs (h3: dense FP16 / 3, x6: dense BF16 / 6, bf16: dense BF16)."""
import bench


def test_kernel_peak_by_operand_planes():
    bf16, h3, x6 = bench.BF16_MFMA_PEAK_TFLOPS, bench.BF16_MFMA_PEAK_TFLOPS / 3, bench.BF16_MFMA_PEAK_TFLOPS / 6
    cases = {
        "conv1d_x6_kernel<6, 2, 2, 8, 2, false, 2, false, true>": h3,
        "conv1d_x6_kernel<6, 2, 2, 8, 1, false, 4, true, true>": bf16,
        "conv1d_x6_kernel<6, 1, 1, 8, 3, false, 1, false, false>": x6,
        "resunit_x6_kernel<6, 1, 1, 8, 2, 2>": h3,
        "resunit_x6_kernel<6, 1, 1, 8, 1, 2>": bf16,
        "resunit_rr_kernel<96, 2, 1>": h3,
        "resunit_strip_kernel<3>": h3,
        "resunit_x6_kernel<3, 1, 1, 8, 3, 2>": x6,
        "resunit_w16_kernel<3, 2, true>": x6,
        "resunit_w16_kernel<1, 2, true>": bf16,
        "lstm_seq2_x6_kernel<12, 3, 2>": x6,
        "lstm_seq2_x6_kernel<12, 2, 1>": h3,
        "pw_presplit_x6_kernel": x6,
        "pw_presplit_kernel": h3,
        "conv1d_mfma_kernel<3, 1, 4, 4, 4>": bench.FP32_MFMA_PEAK_TFLOPS,
    }
    for name, peak in cases.items():
        got = bench.kernel_peak(name)[0]
        assert abs(got - peak) < 1e-9, (name, got, peak)


def test_committed_pmc_summaries_are_readable(tmp_path):
    """bench.py reads the newest profiles/*pmc_traffic.json for the roofline's `traffic`: every committed summary has
    the tools/pmc_summary.py layout ({"kernels": {name: {"traffic_bytes_corrected", ...}}}); a summary is used only
    when its `lib_digest` is the running library's (bc_build_digest), never for other kernel code."""
    import glob
    import json
    import os

    files = sorted(glob.glob(os.path.join(os.path.dirname(bench.__file__), "profiles", "*pmc_traffic.json")))
    assert files
    for f in files:
        d = json.load(open(f))
        assert isinstance(d.get("kernels"), dict), f
        for name, v in d["kernels"].items():
            assert "traffic_bytes_corrected" in v, (f, name)
    k = "conv1d_x6_kernel<6, 2, 2, 8, 3, false, 1, false, true>"
    for i, dig in enumerate(("a" * 64, "b" * 64)):
        (tmp_path / f"r0{i}_pmc_traffic.json").write_text(json.dumps(
            {"lib_digest": dig, "kernels": {k: {"traffic_bytes_corrected": 100.0 + i, "mfma_util": 0.5}}}))
    assert bench.pmc_traffic(k, running="a" * 64, profiles=str(tmp_path)) == (100.0, 0.5, "r00_pmc_traffic.json")
    assert bench.pmc_traffic(k, running="b" * 64, profiles=str(tmp_path))[0] == 101.0
    assert bench.pmc_traffic(k, running="c" * 64, profiles=str(tmp_path)) == (None, None, None)


def test_pmc_summary_takes_the_profiled_benchs_digest(tmp_path):
    """tools/pmc_summary.py stamps a summary with the digest the profiled bench printed in its pass logs,
    and with null when the passes disagree or a log has none -- never with the package's current library."""
    import importlib.util
    import json
    import os

    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(bench.REPO, "tools", "pmc_summary.py"))
    ps = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ps)
    d1, d2 = "a" * 64, "b" * 64
    for p in ("FETCH_SIZE", "WRITE_SIZE", "MFMA"):
        (tmp_path / f"{p}.log").write_text("rocprof noise\n" + json.dumps({"metric": "m", "lib_digest": d1}) + "\n")
    assert ps.profiled_digest(str(tmp_path)) == d1
    (tmp_path / "MFMA.log").write_text(json.dumps({"metric": "m", "lib_digest": d2}) + "\n")
    assert ps.profiled_digest(str(tmp_path)) is None
    (tmp_path / "MFMA.log").write_text("crashed before the line\n")
    assert ps.profiled_digest(str(tmp_path)) is None
