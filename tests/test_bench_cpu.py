"""bench.py's host-side logic (no GPU): the timing window's placement across an episode end, the
launch plan, the host-core count for the CPU baseline and the profile/source pinning."""
import bench


def test_window_is_centred_on_an_episode_end():
    for T in (200, 37):
        for K in (1, 5, 20, 199, 200, 2000):
            for pre in (0, 3, 25, 205, 2200):
                s = bench.window_setup_steps(T, K, pre)
                assert 0 <= s < T
                assert (s + pre + K // 2) % T == 0


def test_launch_plan_covers_exactly_k_steps():
    assert bench.launch_plan(20, 200) == [20]
    assert bench.launch_plan(2000, 200) == [200] * 10
    assert bench.launch_plan(450, 200) == [200, 200, 50]
    assert sum(bench.launch_plan(1234, 97)) == 1234


def test_host_cores_and_aggregate():
    cores, detail = bench.host_cores()
    assert cores >= 1 and "os.cpu_count()" in detail
    assert bench.aggregate_rate(4, 65536, 8, 20, 2.0) == 4 * 65536 * 8 * 20 / 2.0
    assert bench.shard_offset(3, 65536) == 3 * 65536
    assert bench.rank_info({}) == (1, 0, 0)
    assert bench.rank_info({"WORLD_SIZE": "8", "RANK": "5", "LOCAL_RANK": "5"}) == (8, 5, 5)


def test_profiles_are_pinned_to_the_kernel_sources(tmp_path, monkeypatch):
    sha = bench.source_sha()
    assert len(sha) == 16
    # an entry from other sources is not reported
    assert bench.load_profile("no_such_tag") is None


def test_step_roofline_names_the_binding_resource(monkeypatch):
    """roofline.valu = SQ_INSTS_VALU per launch / kernel time against 1,024 SIMDs x 1.2 G wave64-VALU/s;
    `bound` is the larger of the VALU and HBM fractions, both reported."""
    prof = {"avg_ns": 50_000.0, "bytes_per_launch": 5.8e7, "steps_per_launch": 20,
            "sq": {"SQ_INSTS_VALU": 1.8e7, "SQ_WAVES": 1024.0, "SQ_WAVE_CYCLES": 2.8e7, "SQ_INSTS_LDS": 1.5e6,
                   "SQ_WAIT_ANY": 7e6}}
    monkeypatch.setattr(bench, "load_profile", lambda tag: prof)
    m = dict(achieved_gbs=1000.0, kernel_ms=0.05, launches=1, steps_per_launch=20, bytes_per_launch=5.8e7,
             bytes_per_env_step=44.0, host_fixed_us=14.0)
    r = bench.step_roofline(m, "medium", 8, "greedy", "fused", 65536)
    want = 1.8e7 / 50e-6 / 1e9 / (1024 * 1.2)
    assert r["valu"]["frac"] == r["valu_frac"] and abs(r["valu_frac"] - want) < 1e-12
    assert r["frac"] == r["hbm_frac"] == 1000.0 / 8000.0 and r["unit"] == "GB/s"
    assert r["bound"] == "valu" and r["valu_frac"] > r["hbm_frac"]
    assert abs(r["issue"]["single_wave_issue_occupancy"] - 1.8e7 / 2.8e7) < 1e-12
    monkeypatch.setattr(bench, "load_profile", lambda tag: None)
    r = bench.step_roofline(m, "medium", 8, "greedy", "fused", 65536)
    assert r["bound"] == "hbm" and r["valu"] is None
