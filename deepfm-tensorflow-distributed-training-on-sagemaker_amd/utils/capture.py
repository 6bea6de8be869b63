"""One lock between HIP graph captures and the threads that issue GPU work beside them.

The training thread captures multi-step graphs (models/runner.py ``graph_capture``) while the
streamed input's fill thread issues its host-to-device copies, the compact values' expand kernel
and event records on its own copy streams (data/pipeline.py ``_DeviceFeeder``).  Captures use
HIP's thread-local mode, but a fill-thread call that landed inside a capture still invalidated
it now and then (hipErrorStreamCaptureInvalidated at the capture's end, one-process GPU suite
only).  Both sides hold this lock instead: a capture waits for an in-flight batch issue (tens of
microseconds), and the fill thread waits for a capture (captures happen once per run layout)."""
import threading

CAPTURE_LOCK = threading.RLock()
