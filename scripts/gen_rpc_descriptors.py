"""Write ``determined_1_amd/rpc/api_v1.binpb``: the FileDescriptorSet of the
``determined.api.v1.Determined`` service and every message it references, taken from the
reference's compiled image (``proto/buf.image.bin``, a ``google.protobuf.FileDescriptorSet``) with
comments/source info stripped.  It is the wire contract a client generated from the reference's
``api.proto`` speaks; ``rpc/descriptors.py`` builds the request/response classes from it at import
(pure protobuf: no protoc in this image).

    python scripts/gen_rpc_descriptors.py [/root/reference/proto/buf.image.bin]
"""
import os
import sys

from google.protobuf import descriptor_pb2

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/proto/buf.image.bin"
DST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "determined_1_amd", "rpc",
                   "api_v1.binpb")


def main() -> None:
    fds = descriptor_pb2.FileDescriptorSet()
    with open(SRC, "rb") as f:
        fds.ParseFromString(f.read())
    by_name = {f.name: f for f in fds.file}
    keep, order = set(), []

    def visit(name: str) -> None:  # dependencies first, as DescriptorPool.Add requires
        if name in keep:
            return
        keep.add(name)
        for dep in by_name[name].dependency:
            visit(dep)
        order.append(name)

    visit("determined/api/v1/api.proto")
    out = descriptor_pb2.FileDescriptorSet()
    for name in order:
        fd = out.file.add()
        fd.CopyFrom(by_name[name])
        fd.ClearField("source_code_info")
    with open(DST, "wb") as f:
        f.write(out.SerializeToString(deterministic=True))
    print(f"{DST}: {len(order)} files, {os.path.getsize(DST)} bytes")


if __name__ == "__main__":
    main()
