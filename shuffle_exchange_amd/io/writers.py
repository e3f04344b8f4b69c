"""Simple file writers with the FastFileWriter interface (reference io/py_file_writer.py,
io/mock_file_writer.py)."""
import io


class PyFileWriter(io.BufferedWriter):
    def __init__(self, file_path):
        super().__init__(io.FileIO(file_path, "wb"))
        self.file_path = file_path

    def file_path(self):  # noqa: F811 - reference exposes it as a method too
        return self.file_path


class MockFileWriter(io.RawIOBase):
    """Counts bytes, writes nothing (measures serialisation cost without I/O)."""

    def __init__(self, file_path=None):
        self.num_bytes = 0
        self.num_writes = 0
        self.path = file_path

    def writable(self):
        return True

    def write(self, b):
        n = len(memoryview(b).cast("B"))
        self.num_bytes += n
        self.num_writes += 1
        return n
