module github.com/anuragsarkar97/crdt/go/crdt

go 1.18
