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
