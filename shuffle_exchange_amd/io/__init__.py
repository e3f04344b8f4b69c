"""File writers for checkpoints (reference deepspeed/io): FastFileWriter (pinned double-buffered
async writes through the C++ AIO engine), PyFileWriter (plain buffered), MockFileWriter (tests)."""
from .fast_file_writer import FastFileWriter, FastFileWriterConfig  # noqa: F401
from .writers import MockFileWriter, PyFileWriter  # noqa: F401
