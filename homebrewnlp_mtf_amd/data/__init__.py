"""Input side: native TFRecord runtime bindings (``native``), TFRecord / Example IO (``tfrecord``), the text pipeline
(``pipeline``) and the video / jannet pipeline (``video``)."""
