"""GPU-loss health signalling, the Python mirror of the Go
batcher's healthMonitor (go/src/gpu/cache_impl.go): a device-level library
failure (RL_E_HIP, RL_E_COMM, RL_E_INTERNAL) fails the server's health check
once, the next success marks it OK, as the reference's Redis pool does on its
connections (src/redis/driver_impl.go:31-52); request-level failures do not
touch it."""
from ratelimit_amd import abi
from ratelimit_amd._lib import RedisError
from ratelimit_amd.limiter import HealthMonitor


class FakeServer:
    def __init__(self):
        self.calls = []

    def health_check_fail(self):
        self.calls.append("fail")

    def health_check_ok(self):
        self.calls.append("ok")


def _err(st):
    return RedisError("gpu: x [%s]" % abi.STATUS_NAMES[st], st)


def test_device_failure_fails_once_and_recovers():
    srv = FakeServer()
    h = HealthMonitor(srv)
    h.observe(None)
    assert srv.calls == []  # healthy stays quiet
    h.observe(_err(abi.RL_E_HIP))
    h.observe(_err(abi.RL_E_HIP))
    h.observe(_err(abi.RL_E_COMM))
    assert srv.calls == ["fail"]
    h.observe(None)
    h.observe(None)
    assert srv.calls == ["fail", "ok"]
    h.observe(_err(abi.RL_E_INTERNAL))
    assert srv.calls == ["fail", "ok", "fail"]


def test_request_failures_leave_health_alone():
    srv = FakeServer()
    h = HealthMonitor(srv)
    for st in (abi.RL_E_INVALID, abi.RL_E_TABLE_FULL, abi.RL_E_ARENA_FULL, abi.RL_E_CAPACITY, abi.RL_E_TIME):
        h.observe(_err(st))
    h.observe(RedisError("host-side", None))
    assert srv.calls == []
    h.observe(_err(abi.RL_E_HIP))
    h.observe(_err(abi.RL_E_TIME))  # (still unhealthy: a request failure is no recovery)
    assert srv.calls == ["fail"] and h.unhealthy


def test_no_server_no_calls():
    HealthMonitor(None).observe(_err(abi.RL_E_HIP))
