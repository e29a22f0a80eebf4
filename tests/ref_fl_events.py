"""Test infrastructure: the report handler of the reference node restated
(``apps/node/src/app/main/events/model_centric/fl_events.py:237-271``), with its message fields
(``core/codes.py``).  The diff is decoded EXACTLY as the handler does it --
``base64.b64decode(data.get(CYCLE.DIFF, None).encode())`` -- through this module's ``base64`` name,
which ``pygrid_amd.node.install(report_module=...)`` replaces.  ``processes`` stands for
``controller.processes`` (``fl_controller.py:184-194``: ``submit_diff`` ->
``cycle_manager.submit_worker_diff``); the test sets it.  Only tests import this."""
import base64
import traceback

WORKER_ID, KEY, DIFF, STATUS, SUCCESS, ERROR = "worker_id", "request_key", "diff", "status", "success", "error"
REPORT = "model-centric/report"

processes = None


def report(message: dict, socket=None) -> dict:
    data = message["data"]
    response = {}
    try:
        worker_id = data.get(WORKER_ID, None)
        request_key = data.get(KEY, None)
        diff = base64.b64decode(data.get(DIFF, None).encode())
        processes.submit_diff(worker_id, request_key, diff)
        response[STATUS] = SUCCESS
    except Exception as e:  # noqa: BLE001 -- the reference's handler returns the error text
        response[ERROR] = str(e) + traceback.format_exc()
    return {"type": REPORT, "data": response}
