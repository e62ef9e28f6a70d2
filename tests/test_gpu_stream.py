"""stream_of() (the raw current-stream accessor every launch uses) names the same HIP stream as
torch's public API, on the default stream and inside a side-stream context."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wh():
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import warehouse

    return warehouse


def test_stream_of_matches_torch_current_stream(wh):
    from warehouse import _native as nat

    dev = torch.device("cuda", 0)
    assert nat.stream_of(dev) == torch.cuda.current_stream(dev).cuda_stream
    assert nat.stream_of(torch.device("cuda")) == torch.cuda.current_stream().cuda_stream
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        assert nat.stream_of(dev) == s.cuda_stream
    assert nat.stream_of(dev) == torch.cuda.current_stream(dev).cuda_stream
