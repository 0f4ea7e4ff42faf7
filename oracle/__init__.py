"""ORACLE — test infrastructure, NOT the product.

CPU restatement of the reference's per-frame lip-sync path (Ryukhaan/speech-to-video-mpp, a
VideoReTalking fork): LNet/ENet/DNet forward (nets.py), the flow warp, the mel front end
(audio.py), the GFPGAN / GPEN enhancers (enhancers.py), GPEN's ParseNet (parse.py) and the
mouth-region post-process: cv2 pyramids / resize and the Laplacian blend (post.py).  Each function
cites the reference file:line it restates.

Pinning: nets.py and gpen_ops.py are checked against golden fixtures produced by running the
reference itself in the build container (tests/golden/make_golden.py, tests/test_oracle_golden.py).
audio.py is "parity unpinned": the reference's mel goes through librosa 0.9.2, which is absent
from this image and from the reference tree.  post.py is "parity unpinned" against
cv2 (absent too); it is pinned by hand-computed known answers (tests/test_post_host.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
"""
