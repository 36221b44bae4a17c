"""Console + per-run log file, as the reference CLIs configure it (logging_utils.py:14-63)."""
import logging

_FMT = "[%(asctime)s] %(levelname)8s %(message)s (%(filename)s:%(lineno)d)"


def configure_logging(console_level="WARNING", file_path=None, file_level="INFO", force=False):
    root = logging.getLogger()
    if force:
        for h in list(root.handlers):
            root.removeHandler(h)
    root.setLevel(logging.DEBUG)
    ch = logging.StreamHandler()
    ch.setLevel(console_level)
    ch.setFormatter(logging.Formatter(_FMT, "%Y-%m-%d %H:%M:%S"))
    root.addHandler(ch)
    if file_path:
        fh = logging.FileHandler(file_path, mode="w")
        fh.setLevel(file_level)
        fh.setFormatter(logging.Formatter(_FMT, "%Y-%m-%d %H:%M:%S"))
        root.addHandler(fh)


def get_logger(name):
    return logging.getLogger(name)
