"""MI355X-native Prov-GigaPath slide encoder (drop-in for the reference's ``gigapath`` package
on the slide-encoder path).  See DESIGN.md."""
