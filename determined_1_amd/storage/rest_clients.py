"""Object-store clients over the stores' plain HTTP APIs (no boto3 / google-cloud-storage / hdfs
SDK on this image): S3 (AWS Signature V4, multipart upload for large files), GCS (JSON API with
an OAuth bearer token) and HDFS (WebHDFS).  They implement ``cloud.ObjectClient`` and are what
``S3StorageManager`` / ``GCSStorageManager`` / ``HDFSStorageManager`` use by default (reference
``harness/determined/common/storage/{s3,gcs,hdfs}.py`` over the vendor SDKs).

Every client accepts ``endpoint_url`` so a MinIO / fake-gcs / local WebHDFS endpoint (and the
test fakes in ``tests/test_storage_rest.py``) can stand in for the cloud.
"""
import datetime
import hashlib
import hmac
import os
import urllib.parse
import xml.etree.ElementTree as ET
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Iterator, List, Optional, Tuple

import requests

from determined_1_amd.storage.cloud import ObjectClient

CHUNK = 8 << 20


def _write_stream(resp: requests.Response, dst: str) -> None:
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst, "wb") as f:
        for chunk in resp.iter_content(CHUNK):
            f.write(chunk)


# -------------------------------------------------------------------------------------- S3
def _sha256(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def sigv4_headers(method: str, url: str, region: str, access_key: str, secret_key: str, payload_hash: str,
                  session_token: Optional[str] = None, service: str = "s3",
                  now: Optional[datetime.datetime] = None, extra: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """AWS Signature Version 4 headers for one request (header-based auth)."""
    now = now or datetime.datetime.now(datetime.timezone.utc)
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    date = amz_date[:8]
    u = urllib.parse.urlsplit(url)
    host = u.netloc
    # S3 canonical URI = the path URI-encoded ONCE (RFC 3986 unreserved kept, '/' kept).  ``url`` comes
    # from ``_url`` already encoded, so normalise through unquote (a second quote would turn '%3D'
    # into '%253D' and every key with '=', '+' or a space would fail SignatureDoesNotMatch).
    canon_uri = urllib.parse.quote(urllib.parse.unquote(u.path or "/"), safe="/~-_.")
    q = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    canon_q = "&".join(f"{urllib.parse.quote(k, safe='~-_.')}={urllib.parse.quote(v, safe='~-_.')}"
                       for k, v in sorted(q))
    headers = {"host": host, "x-amz-content-sha256": payload_hash, "x-amz-date": amz_date}
    if session_token:
        headers["x-amz-security-token"] = session_token
    for k, v in (extra or {}).items():
        headers[k.lower()] = v
    signed = ";".join(sorted(headers))
    canon_headers = "".join(f"{k}:{headers[k].strip()}\n" for k in sorted(headers))
    canon = "\n".join([method, canon_uri, canon_q, canon_headers, signed, payload_hash])
    scope = f"{date}/{region}/{service}/aws4_request"
    to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, _sha256(canon.encode())])
    k = _hmac(_hmac(_hmac(_hmac(("AWS4" + secret_key).encode(), date), region), service), "aws4_request")
    sig = hmac.new(k, to_sign.encode(), hashlib.sha256).hexdigest()
    out = {k2: v for k2, v in headers.items() if k2 != "host"}
    out["Authorization"] = f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, SignedHeaders={signed}, Signature={sig}"
    return out


class S3RestClient(ObjectClient):
    NS = "{http://s3.amazonaws.com/doc/2006-03-01/}"

    def __init__(self, bucket: str, access_key: Optional[str] = None, secret_key: Optional[str] = None,
                 endpoint_url: Optional[str] = None, region: Optional[str] = None,
                 session_token: Optional[str] = None, multipart_threshold: int = 64 << 20,
                 part_size: int = 64 << 20) -> None:
        self.bucket = bucket
        self.access_key = access_key or os.environ.get("AWS_ACCESS_KEY_ID", "")
        self.secret_key = secret_key or os.environ.get("AWS_SECRET_ACCESS_KEY", "")
        self.session_token = session_token or os.environ.get("AWS_SESSION_TOKEN")
        self.region = region or os.environ.get("AWS_DEFAULT_REGION", "us-east-1")
        if endpoint_url:  # path-style (MinIO, fakes)
            self.base = endpoint_url.rstrip("/") + "/" + bucket
        else:
            self.base = f"https://{bucket}.s3.{self.region}.amazonaws.com"
        self.multipart_threshold = multipart_threshold
        self.part_size = part_size
        self.session = requests.Session()

    def _url(self, key: str, query: str = "") -> str:
        """Object URL (or the bucket URL for key ""), path-style under an endpoint override."""
        return self.base + "/" + urllib.parse.quote(key, safe="/~-_.") + (("?" + query) if query else "")

    def _req(self, method: str, url: str, data: bytes = b"", stream: bool = False,
             extra: Optional[Dict[str, str]] = None, ok: Tuple[int, ...] = (200,)) -> requests.Response:
        h = sigv4_headers(method, url, self.region, self.access_key, self.secret_key, _sha256(data),
                          self.session_token, extra=extra)
        r = self.session.request(method, url, data=data or None, headers=h, stream=stream, timeout=300)
        if r.status_code not in ok:
            raise IOError(f"S3 {method} {url}: {r.status_code} {r.text[:300]}")
        return r

    def upload_file(self, local: str, key: str) -> None:
        size = os.path.getsize(local)
        if size <= self.multipart_threshold:
            with open(local, "rb") as f:
                self._req("PUT", self._url(key), f.read())
            return
        r = self._req("POST", self._url(key, "uploads="))
        upload_id = ET.fromstring(r.content).find(f"{self.NS}UploadId")
        upload_id = upload_id.text if upload_id is not None else ET.fromstring(r.content).findtext("UploadId")
        etags: List[str] = []
        try:
            with open(local, "rb") as f:
                n = 1
                while True:
                    part = f.read(self.part_size)
                    if not part:
                        break
                    q = f"partNumber={n}&uploadId={urllib.parse.quote(upload_id, safe='')}"
                    pr = self._req("PUT", self._url(key, q), part)
                    etags.append(pr.headers.get("ETag", ""))
                    n += 1
            body = "<CompleteMultipartUpload>" + "".join(
                f"<Part><PartNumber>{i + 1}</PartNumber><ETag>{e}</ETag></Part>" for i, e in enumerate(etags)
            ) + "</CompleteMultipartUpload>"
            self._req("POST", self._url(key, f"uploadId={urllib.parse.quote(upload_id, safe='')}"), body.encode())
        except Exception:
            self._req("DELETE", self._url(key, f"uploadId={urllib.parse.quote(upload_id, safe='')}"), ok=(200, 204))
            raise

    def list(self, prefix: str) -> Iterator[str]:
        token = None
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if token:
                q["continuation-token"] = token
            r = self._req("GET", self._url("", urllib.parse.urlencode(q)))
            root = ET.fromstring(r.content)
            ns = self.NS if root.tag.startswith(self.NS) else ""
            for c in root.findall(f"{ns}Contents"):
                yield c.findtext(f"{ns}Key")
            if root.findtext(f"{ns}IsTruncated") != "true":
                return
            token = root.findtext(f"{ns}NextContinuationToken")

    def download_dir(self, prefix: str, local_dir: str) -> None:
        prefix = prefix.rstrip("/") + "/" if prefix else ""
        keys = [k for k in self.list(prefix)]

        def get(k: str) -> None:
            dst = os.path.join(local_dir, os.path.relpath(k, prefix) if prefix else k)
            if k.endswith("/"):
                os.makedirs(dst, exist_ok=True)
                return
            _write_stream(self._req("GET", self._url(k), stream=True), dst)

        with ThreadPoolExecutor(8) as ex:
            list(ex.map(get, keys))

    def delete_prefix(self, prefix: str) -> None:
        prefix = prefix.rstrip("/") + "/" if prefix else ""
        keys = list(self.list(prefix))
        with ThreadPoolExecutor(8) as ex:
            list(ex.map(lambda k: self._req("DELETE", self._url(k), ok=(200, 204)), keys))


# ------------------------------------------------------------------------------------- GCS
class GCSRestClient(ObjectClient):
    """GCS JSON API.  Auth: ``token`` / ``$GOOGLE_OAUTH_ACCESS_TOKEN`` or, on GCE, the metadata
    server's service-account token."""

    def __init__(self, bucket: str, endpoint_url: Optional[str] = None, token: Optional[str] = None) -> None:
        self.bucket = bucket
        self.base = (endpoint_url or "https://storage.googleapis.com").rstrip("/")
        self._token = token or os.environ.get("GOOGLE_OAUTH_ACCESS_TOKEN")
        self.session = requests.Session()

    def _auth(self) -> Dict[str, str]:
        if not self._token:
            try:
                r = requests.get("http://metadata.google.internal/computeMetadata/v1/instance/service-accounts/"
                                 "default/token", headers={"Metadata-Flavor": "Google"}, timeout=5)
                self._token = r.json()["access_token"]
            except (requests.RequestException, KeyError, ValueError) as e:
                raise IOError(f"GCS: no access token (set GOOGLE_OAUTH_ACCESS_TOKEN): {e}") from e
        return {"Authorization": f"Bearer {self._token}"}

    def _obj(self, key: str) -> str:
        return f"{self.base}/storage/v1/b/{self.bucket}/o/{urllib.parse.quote(key, safe='')}"

    def upload_file(self, local: str, key: str) -> None:
        url = f"{self.base}/upload/storage/v1/b/{self.bucket}/o?uploadType=media&name={urllib.parse.quote(key, safe='')}"
        with open(local, "rb") as f:
            r = self.session.post(url, data=f, headers=dict(self._auth(), **{"Content-Type": "application/octet-stream"}),
                                  timeout=600)
        if r.status_code != 200:
            raise IOError(f"GCS upload {key}: {r.status_code} {r.text[:300]}")

    def list(self, prefix: str) -> Iterator[str]:
        token = None
        while True:
            params = {"prefix": prefix}
            if token:
                params["pageToken"] = token
            r = self.session.get(f"{self.base}/storage/v1/b/{self.bucket}/o", params=params, headers=self._auth(),
                                 timeout=60)
            if r.status_code != 200:
                raise IOError(f"GCS list {prefix}: {r.status_code} {r.text[:300]}")
            j = r.json()
            for it in j.get("items", []):
                yield it["name"]
            token = j.get("nextPageToken")
            if not token:
                return

    def download_dir(self, prefix: str, local_dir: str) -> None:
        prefix = prefix.rstrip("/") + "/" if prefix else ""
        for k in list(self.list(prefix)):
            dst = os.path.join(local_dir, os.path.relpath(k, prefix) if prefix else k)
            if k.endswith("/"):
                os.makedirs(dst, exist_ok=True)
                continue
            r = self.session.get(self._obj(k), params={"alt": "media"}, headers=self._auth(), stream=True, timeout=600)
            if r.status_code != 200:
                raise IOError(f"GCS get {k}: {r.status_code}")
            _write_stream(r, dst)

    def delete_prefix(self, prefix: str) -> None:
        prefix = prefix.rstrip("/") + "/" if prefix else ""
        for k in list(self.list(prefix)):
            r = self.session.delete(self._obj(k), headers=self._auth(), timeout=60)
            if r.status_code not in (200, 204, 404):
                raise IOError(f"GCS delete {k}: {r.status_code}")


# ------------------------------------------------------------------------------------ HDFS
class WebHDFSClient(ObjectClient):
    """WebHDFS REST (``http://<namenode>:9870/webhdfs/v1``): CREATE/OPEN follow the namenode's
    redirect to a datanode, as the protocol requires."""

    def __init__(self, url: str, user: Optional[str] = None) -> None:
        self.base = url.rstrip("/") + "/webhdfs/v1"
        self.user = user or os.environ.get("HADOOP_USER_NAME") or os.environ.get("USER", "root")
        self.session = requests.Session()

    def _u(self, path: str, op: str, **params: str) -> str:
        q = dict(params, op=op, **{"user.name": self.user})
        return f"{self.base}/{urllib.parse.quote(path.lstrip('/'), safe='/')}?{urllib.parse.urlencode(q)}"

    def upload_file(self, local: str, key: str) -> None:
        r = self.session.put(self._u(key, "CREATE", overwrite="true"), allow_redirects=False, timeout=60)
        if r.status_code == 307:
            with open(local, "rb") as f:
                r = self.session.put(r.headers["Location"], data=f, timeout=600)
        if r.status_code != 201:
            raise IOError(f"WebHDFS CREATE {key}: {r.status_code} {r.text[:300]}")

    def _walk(self, path: str) -> Iterator[str]:
        r = self.session.get(self._u(path, "LISTSTATUS"), timeout=60)
        if r.status_code == 404:
            return
        if r.status_code != 200:
            raise IOError(f"WebHDFS LISTSTATUS {path}: {r.status_code}")
        for st in r.json()["FileStatuses"]["FileStatus"]:
            child = path.rstrip("/") + "/" + st["pathSuffix"]
            if st["type"] == "DIRECTORY":
                yield from self._walk(child)
            else:
                yield child

    def download_dir(self, prefix: str, local_dir: str) -> None:
        for p in list(self._walk(prefix)):
            r = self.session.get(self._u(p, "OPEN"), stream=True, timeout=600)
            if r.status_code != 200:
                raise IOError(f"WebHDFS OPEN {p}: {r.status_code}")
            _write_stream(r, os.path.join(local_dir, os.path.relpath(p, prefix.rstrip("/"))))

    def delete_prefix(self, prefix: str) -> None:
        r = self.session.delete(self._u(prefix, "DELETE", recursive="true"), timeout=60)
        if r.status_code not in (200, 404):
            raise IOError(f"WebHDFS DELETE {prefix}: {r.status_code}")
